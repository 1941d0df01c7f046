# Round 2, call AD: full GPU suite + smoke on the build whose exact dispatch takes the 8-B
# chain-hopping forms for odd widths.
set -o pipefail
mkdir -p gpurun_out/r02ad
O=gpurun_out/r02ad
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
echo all-done
