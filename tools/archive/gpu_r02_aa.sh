# Round 2, call AA: the text loader on the GPU box's host (16-CPU share), then the executables'
# tests that go through it (mpiexec, y files) and the full GPU suite.
set -o pipefail
mkdir -p gpurun_out/r02aa
O=gpurun_out/r02aa
timeout -k 10 300 python -u tools/load_bench.py 16384 16384 1,4,8,16 /tmp/mvg_load_bench > $O/load_bench.jsonl 2> $O/load_bench.err || { tail -20 $O/load_bench.err; exit 1; }
cat $O/load_bench.jsonl
rm -rf /tmp/mvg_load_bench
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
echo all-done
