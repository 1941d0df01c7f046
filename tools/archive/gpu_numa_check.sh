set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -k "shared or bench_two" -x -v --timeout 200 --timeout-method thread > gpurun_out/numa_test.log 2>&1 || { tail -30 gpurun_out/numa_test.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/numa_test.log
MVG_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --no-cpu-baseline --no-configs > gpurun_out/numa_b1.json 2> gpurun_out/numa_b1.err || { tail -20 gpurun_out/numa_b1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/numa_b1.json')); print(d['value'], d['end_to_end'])"
