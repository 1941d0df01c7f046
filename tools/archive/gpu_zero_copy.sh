set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/zero_copy_probe.py > gpurun_out/zero_copy.jsonl 2> gpurun_out/zero_copy.err || { tail -20 gpurun_out/zero_copy.err; exit 1; }
cat gpurun_out/zero_copy.jsonl
