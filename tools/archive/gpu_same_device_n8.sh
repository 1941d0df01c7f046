# The driver's scaling invocation (torch.distributed.run, N = 4 and 8, default steps) rehearsed
# with every rank on GPU 0 (MVG_SAME_DEVICE=1: RCCL over loopback sockets; timings mean nothing).
set -o pipefail
mkdir -p gpurun_out
for n in 4 8; do
MVG_SAME_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2954$n bench.py --gpus $n > gpurun_out/same$n.json 2> gpurun_out/same$n.err || { tail -30 gpurun_out/same$n.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/same$n.json')); print($n, d['value'], d['config']['R'], d['config']['bytes_per_step'], {k: (v['mean_s'] if isinstance(v, dict) else v) for k, v in d['end_to_end'].items() if k not in ('semantics', 'roofline')})"
done
