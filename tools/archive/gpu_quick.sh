# Quick GPU check: parity tests, then the default bench and forced-exchange benches (N = 1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
for ring in 1 8; do for a in rowwise colwise blockwise; do
MVG_XRING=$ring MVG_ALWAYS_COLLECT=1 timeout -k 10 300 python bench.py --alg $a --no-cpu-baseline --no-e2e --steps 100 > gpurun_out/bench_x_$a.json 2>> gpurun_out/bench_x.err || { tail gpurun_out/bench_x.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_x_$a.json')); print('ring$ring $a', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done; done
