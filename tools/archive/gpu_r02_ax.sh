# Round 2, call AX: the dispatch with XCD-ordered row-block forms on tall shapes (auto against
# the forms it replaces), then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out/r02ax
O=gpurun_out/r02ax
S=cfg3_g8_strip_65536x8192,cfg4_block_65536x32768,cfg3_g4_strip_65536x16384,cfg3_g1_65536sq,cfg2_16384sq,524288x4096,262144x5120,131072x3072,1048576x2048,65536x4200,32768x8192,cfg5_shard_524288x512
V='rowblk_w4_r2_u8$,rowblk_w8_r2_u4$,vec_l64_r2_u4_nt1_o7$'
timeout -k 10 600 python -u tools/sweep_variants.py 5 $S $V > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
echo all-done
