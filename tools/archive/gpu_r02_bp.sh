# Round 2, call BP: the clean-built final library — GPU suite and smoke() as the driver runs them.
set -o pipefail
mkdir -p gpurun_out/r02bp
O=gpurun_out/r02bp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo all-done
