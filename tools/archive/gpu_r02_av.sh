# Round 2, call AV: XCD-remapped row-block forms against the dispatch's plain ones on tall
# long-row shapes (config 3 / 4 shards and their neighbours), 7 interleaved rounds each.
set -o pipefail
mkdir -p gpurun_out/r02av
O=gpurun_out/r02av
S=cfg3_g8_strip_65536x8192,cfg3_g4_strip_65536x16384,cfg4_block_65536x32768,cfg3_g1_65536sq,mid_524288x4096,mid_1048576x2048,131072x8192,131072x16384,131072x32768,262144x8192,32768x16384,32768x32768,32768x8192,cfg4_full_131072sq
V='rowblk_w4_r2_u8$,rowblk_w4_r2_u8_xcd$,rowblk_w8_r2_u4$,rowblk_w8_r2_u4_xcd$'
timeout -k 10 900 python -u tools/sweep_variants.py 7 $S $V > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
