# Round 2, call BN: XCD-contiguous workgroup order for the panel exact kernel (panel_*_xcd)
# against the plain order, on the panel dispatch's shapes, P = 256, 9 rounds.
set -o pipefail
mkdir -p gpurun_out/r02bn
O=gpurun_out/r02bn
S=cfg2_16384sq,ref_10200sq,cfg3_g8_strip_65536x8192,cfg4_block_65536x32768,tall_262144x4096,tall_131072x16384,mid_6144x4096
timeout -k 10 600 python -u tools/panel_probe.py 9 $S 256 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
echo all-done
