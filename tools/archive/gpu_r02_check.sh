# Round 2 check: GPU parity tests (incl. the rank-mode back-to-back test), smoke, bench, and the
# reference CPU sweep with enforced CPU placement.
set -o pipefail
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"
echo "== pytest gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
grep smoke gpurun_out/smoke.log
echo "== bench"; timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== cpu sweep"; timeout -k 10 600 python tools/cpu_ref_sweep.py > gpurun_out/cpu_ref_sweep.jsonl 2> gpurun_out/cpu_ref_sweep.err || { tail gpurun_out/cpu_ref_sweep.err; exit 1; }
cat gpurun_out/cpu_ref_sweep.jsonl
