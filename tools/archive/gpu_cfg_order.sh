# Does the order of the configs section change configs 4/5 (allocation after frees)? Plus the
# config-2-only rocprofv3 kernel stats of the bench's main measurement.
set -o pipefail
mkdir -p gpurun_out
for order in "3,4,5" "5,3,4" "4" "5"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 10 --configs $order > gpurun_out/order.json 2> gpurun_out/order.err || { tail gpurun_out/order.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/order.json')); print('$order', [(c['config'], c['kernel_ms'], c['kernel_frac']) for c in d['configs']])"
done
R=$PWD; cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-configs > $R/gpurun_out/prof2_bench.json 2> $R/gpurun_out/prof2.err || { tail $R/gpurun_out/prof2.err; exit 1; }
cd $R; head -2 gpurun_out/prof2/run_kernel_stats.csv; cat gpurun_out/prof2_bench.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['roofline']['kernel_ms'])"
