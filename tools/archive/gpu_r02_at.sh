# Round 2, call AT: the tree's line-aligned row-pair form (rows off the 128-B lines) — parity
# tests over every variant, then the sweep against the current dispatch on off-line shapes.
set -o pipefail
mkdir -p gpurun_out/r02at
O=gpurun_out/r02at
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
timeout -k 10 600 python -u tools/sweep_variants.py 3 16384x16386,16384x16383,10200x10200,4200x4200,65536x8191,16384x16384,1800x1800,7800x7800,65536x4200,2048x65535 rowlines,rowblk_w4_r2_u8$,rowblk_w4_r2_u8_xcd$,rowblk_w8_r2_u4$,rowblk_w2_r2_u4$ > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
