# Round-4 final check on one MI355X (gpurun, repo root): the GPU test suite, smoke(), the
# driver's N = 1 bench under rocprofv3's kernel trace, then the exact-context probe. Output in
# gpurun_out/$OUT; each GPU step under its own time limit, the first failure ends the script.
set -o pipefail
OUT=gpurun_out/${OUT:-f4a}
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
echo "== bench N=1 under rocprofv3"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o run -- \
    python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/bench.json 2> $ROOT/$OUT/bench.err || { tail $ROOT/$OUT/bench.err; exit 1; }
cd $ROOT && python3 tools/rocprof_by_grid.py $OUT/prof --out $OUT/kernel_by_grid.csv
tail -c 200 $OUT/bench.json
echo "== bench N=1, the driver's command untraced"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_untraced.json 2> $OUT/bench_untraced.err || { tail $OUT/bench_untraced.err; exit 1; }
tail -c 200 $OUT/bench_untraced.json
echo "== exact context probe"
timeout -k 10 150 python -u tools/probes/exact_context_probe.py engine 16384 16384 50 > $OUT/probe.jsonl 2> $OUT/probe.err || exit $?
timeout -k 10 200 python -u tools/probes/exact_context_probe.py queues 16384 16384 30 >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit $?
