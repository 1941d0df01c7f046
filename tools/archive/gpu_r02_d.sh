# Round 2, call D: the whole GPU suite with the exact mode (kernels, engine, executables under
# mpiexec), then the default bench (now with its `exact` section) and the exact kernel under
# rocprofv3 --kernel-trace --stats.
set -o pipefail
mkdir -p gpurun_out/r02d
O=gpurun_out/r02d
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
echo "== bench"
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], json.dumps(d['exact']))"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "== rocprofv3 stats (exact section only timed separately)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_exact -o run -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-configs --steps 100 --warmup 10 > $R/$O/prof_exact.json 2> $R/$O/prof_exact.err || { tail -20 $R/$O/prof_exact.err; exit 1; }
cat $R/$O/prof_exact/run_kernel_stats.csv
echo all-done
