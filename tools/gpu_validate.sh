# Whole-build check on one MI355X (run through gpurun from the repo root): the GPU test suite,
# smoke(), and the driver's bench command under rocprofv3's kernel trace. Output in
# gpurun_out/validate/ (bench.json, kernel_stats.csv, kernel_trace.csv, logs).
set -o pipefail
OUT=gpurun_out/validate
mkdir -p $OUT
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
echo "== bench under rocprofv3"
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o run -- \
    python3 $ROOT/bench.py > $ROOT/$OUT/bench.json 2> $ROOT/$OUT/bench.err || { tail $ROOT/$OUT/bench.err; exit 1; }
cd $ROOT
tail -c 400 $OUT/bench.json
