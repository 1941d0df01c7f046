# Round 2, call AE: the tree kernels' 16-B forms on odd lda / 8-B offset views (unaligned vector
# loads) — parity tests, then the variant sweep on odd-width shapes beside the 8-B forms.
set -o pipefail
mkdir -p gpurun_out/r02ae
O=gpurun_out/r02ae
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
timeout -k 10 700 python -u tools/sweep_variants.py 3 16384x16383,65536x8191,4096x16383,1200x60001,10200x1275,4200x525,524288x511,2048x65535,16384x16384 vec,rowblk,scl > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
