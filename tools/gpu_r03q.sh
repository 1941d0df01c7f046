set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03q
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-e2e --no-cpu-baseline --no-loader > gpurun_out/r03q/bench_multi16.json 2> gpurun_out/r03q/bench_multi16.err
