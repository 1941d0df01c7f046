# Multi-vector GEMV: every-variant parity tests, then the variant sweep (tools/multi_bench.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k multi_vector -x -q --timeout 120 --timeout-method thread > gpurun_out/multi_test.log 2>&1 || { tail -30 gpurun_out/multi_test.log; exit 1; }
tail -2 gpurun_out/multi_test.log
timeout -k 10 900 python -u tools/multi_bench.py $MB_SHAPES > gpurun_out/multi_sweep.jsonl 2> gpurun_out/multi_sweep.err || { tail -20 gpurun_out/multi_sweep.err; exit 1; }
wc -l gpurun_out/multi_sweep.jsonl
