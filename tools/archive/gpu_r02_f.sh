# Round 2, call F: register-staged exact variants — exact parity, then the sweep.
set -o pipefail
mkdir -p gpurun_out/r02f
O=gpurun_out/r02f
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1; rc=$?
tail -3 $O/pytest_exact.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_exact.log | head -20; exit $rc; }
timeout -k 10 500 python -u tools/sweep_exact.py 3 > $O/sweep_exact.jsonl 2> $O/sweep_exact.err || { tail -20 $O/sweep_exact.err; exit 1; }
echo all-done
