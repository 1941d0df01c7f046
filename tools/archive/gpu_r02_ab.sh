# Round 2, call AB: the driver's N = 8 command on the current build (exact sections, exact
# configs, chain-hopping dispatch) with every rank on GPU 0 (MVG_SAME_DEVICE=1; timings mean
# nothing, the point is that every path runs to one valid JSON line).
set -o pipefail
mkdir -p gpurun_out/r02ab
O=gpurun_out/r02ab
start=$(date +%s)
MVG_SAME_DEVICE=1 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29548 bench.py --gpus 8 > $O/same8.json 2> $O/same8.err || { tail -30 $O/same8.err; exit 1; }
echo "elapsed $(( $(date +%s) - start )) s"
python -c "import json; d=json.load(open('$O/same8.json')); print(d['n_gpus'], d['value'], d['exact']['kernel'], d['exact']['max_rel_vs_tree'], [(c['config'], c.get('grid'), c['exact']['kernel'], c['exact']['max_rel_vs_tree']) for c in d['configs']])"
echo all-done
