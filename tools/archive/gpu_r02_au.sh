# Round 2, call AU: the tree dispatch with the line-aligned row-pair form for off-line rows —
# the off-line sweep (auto against the previous choices), then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out/r02au
O=gpurun_out/r02au
timeout -k 10 600 python -u tools/sweep_variants.py 3 16384x16386,16384x16383,10200x10200,7800x7800,65536x8191,16384x16384,65536x8192 rowlines_w8_u4_x0$,rowblk_w4_r2_u8$,rowblk_w4_r2_u8_xcd$,rowblk_w8_r2_u4$ > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
echo all-done
