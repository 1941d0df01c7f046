# Round 2, call AL: the final exact dispatch — exact tests and the sweep over every shape.
set -o pipefail
mkdir -p gpurun_out/r02al
O=gpurun_out/r02al
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
timeout -k 10 900 python -u tools/sweep_exact.py 3 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
