# Round 2, call C: the bit-exact kernels — parity first (tests/test_gpu_exact.py), then a sweep
# of the exact variants against the tree-summed GEMV.
set -o pipefail
mkdir -p gpurun_out/r02c
O=gpurun_out/r02c
echo "== exact parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1; rc=$?
tail -40 $O/pytest_exact.log
[ $rc -eq 0 ] || exit $rc
echo "== exact sweep"
timeout -k 10 500 python -u tools/sweep_exact.py 3 > $O/sweep_exact.jsonl 2> $O/sweep_exact.err || { tail -20 $O/sweep_exact.err; exit 1; }
cat $O/sweep_exact.jsonl
echo all-done
