# Round-4: exact forms under sustained load, then the GPU test suite and smoke() (gpurun, repo root).
set -o pipefail
OUT=gpurun_out/${OUT:-t4a}
mkdir -p $OUT
echo "== sustained exact forms"
timeout -k 10 300 python -u tools/probes/exact_context_probe.py sustained 16384 16384 100 > $OUT/sustained_16384.jsonl 2> $OUT/sustained.err || exit $?
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
