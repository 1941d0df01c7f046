# Round 2, call BJ: the panel layout on fewer rows (2048 .. 6143, outside the current panel
# dispatch): the product's panel variants (8 and 16 lanes per row) against the row-major exact
# dispatch, P = 128 / 256.
set -o pipefail
mkdir -p gpurun_out/r02bj
O=gpurun_out/r02bj
S=ref_4200sq,ref_5400sq,mid_4096x16384,mid_4096x32768,mid_2048x65536,mid_6144x2048
timeout -k 10 600 python -u tools/panel_probe.py 7 $S 128,256 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
echo all-done
