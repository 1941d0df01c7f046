# Multi-rank rehearsal on a one-GPU box (every rank on GPU 0, RCCL over loopback sockets):
# the executables under mpiexec -n 2..4 against the reference's golden y, then bench.py at N = 2
# under torch.distributed.run for all three algorithms.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/same_device_parity.py > gpurun_out/same_device_parity.jsonl 2> gpurun_out/same_device_parity.err || { tail -20 gpurun_out/same_device_parity.jsonl; tail -20 gpurun_out/same_device_parity.err; exit 1; }
tail -1 gpurun_out/same_device_parity.jsonl
for alg in rowwise colwise blockwise; do
MVG_SAME_DEVICE=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --alg $alg --steps 5 --warmup 2 --e2e-iters 2 > gpurun_out/same2_$alg.json 2> gpurun_out/same2_$alg.err || { tail -30 gpurun_out/same2_$alg.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/same2_$alg.json')); print('$alg', d['n_gpus'], d['config']['parallelism'], {k: (v['mean_s'] if isinstance(v, dict) else v) for k, v in d['end_to_end'].items() if k not in ('semantics', 'roofline')})"
done
