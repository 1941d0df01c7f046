# One GPU round: parity tests, smoke, bench, rocprofv3 kernel stats, PMC passes.
set -o pipefail
mkdir -p gpurun_out
df -h /dev/shm /tmp 2>/dev/null | tail -2; free -g | head -2; nproc
echo "== pytest gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
grep smoke gpurun_out/smoke.log
echo "== bench"; timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== rocprof"; R=$PWD; cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err || { tail $R/gpurun_out/prof.err; exit 1; }
cd $R && python3 tools/rocprof_by_grid.py gpurun_out/prof --out gpurun_out/prof_by_grid.csv && head -8 gpurun_out/prof_by_grid.csv
bash tools/gpu_pmc.sh
