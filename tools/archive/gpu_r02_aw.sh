# Round 2, call AW: row-block forms (plain and XCD-remapped) against the dispatch's wave-owns-rows
# forms on tall shapes with 2048 <= K < 8192 and A >= 1 GiB, 7 interleaved rounds each.
set -o pipefail
mkdir -p gpurun_out/r02aw
O=gpurun_out/r02aw
S=524288x4096,262144x4096,131072x4096,65536x4096,65536x4200,262144x6144,131072x6144,65536x6144,524288x2048,1048576x2048,349525x3072,131072x3072,262144x5120
V='rowblk_w4_r2_u8$,rowblk_w4_r2_u8_xcd$,rowblk_w8_r2_u4$,rowblk_w8_r2_u4_xcd$,rowblk_w2_r2_u4$,rowblk_w4_r2_u4$,vec_l64_r2_u4_nt1_o7$,vec_l64_r4_u4_nt1_o5$'
timeout -k 10 900 python -u tools/sweep_variants.py 7 $S $V > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
