# Round 2, call H: the default bench with exact-mode configs, then the driver's N = 4 command
# rehearsed with every rank on GPU 0 (exact exchange over RCCL at 4 ranks).
set -o pipefail
mkdir -p gpurun_out/r02h
O=gpurun_out/r02h
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['exact']['value'], [(c['config'], c['value'], c['kernel_frac'], c['exact']) for c in d['configs']])"
MVG_SAME_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 4 > $O/same4.json 2> $O/same4.err || { tail -30 $O/same4.err; exit 1; }
python -c "import json; d=json.load(open('$O/same4.json')); print(d['n_gpus'], d['value'], d['exact'], [(c['config'], c.get('grid'), c['exact']) for c in d['configs']])"
echo all-done
