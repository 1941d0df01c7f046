# Round 2, call AY: 65536 x 32768 (config 4 block at G = 8) again — XCD order against the plain
# order, 9 interleaved rounds, on two allocations (the shape run twice) plus neighbours.
set -o pipefail
mkdir -p gpurun_out/r02ay
O=gpurun_out/r02ay
S=cfg4_block_65536x32768,65536x32768,131072x16384,32768x32768,cfg3_g8_strip_65536x8192
V='rowblk_w4_r2_u8$,rowblk_w4_r2_u8_xcd$,rowblk_w8_r2_u4_xcd$,rowblk_w4_r2_u8_xq256$,rowblk_w4_r2_u8_xq64$'
timeout -k 10 600 python -u tools/sweep_variants.py 9 $S $V > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
