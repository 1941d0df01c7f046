# Round 2, call AG: longer runs per lane between hops (W = 16) on the chain-bound few-row shapes,
# after the exact parity tests (which cover the new variants).
set -o pipefail
mkdir -p gpurun_out/r02ag
O=gpurun_out/r02ag
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
timeout -k 10 600 python -u tools/sweep_exact.py 3 asym_120x60000,asym_1200x60000,mid_2048x65536,ref_1800sq,mid_4096x32768,ref_10200sq > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
