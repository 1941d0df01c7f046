# Default bench (N = 1) with both CPU baselines, plus its wall time.
set -o pipefail
mkdir -p gpurun_out
t0=$(date +%s)
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - t0 )) s"
cat gpurun_out/bench.json
