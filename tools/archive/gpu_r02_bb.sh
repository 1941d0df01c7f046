# Round 2, call BB: the chain-hopping exact GEMV over a column-panel layout of A
# (tools/micro/panel_hop.hip, tools/panel_probe.py) against the row-major exact dispatch, the
# tree kernel and a plain streaming read; y checked bit for bit against the row-major exact y.
set -o pipefail
mkdir -p gpurun_out/r02bb
O=gpurun_out/r02bb
S=cfg2_16384sq,mid_8192x16384,cfg3_g8_strip_65536x8192,cfg5_shard_524288x512,cfg4_block_65536x32768
timeout -k 10 600 python -u tools/panel_probe.py 5 $S 16,64,128,256,1024,4096 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
echo all-done
