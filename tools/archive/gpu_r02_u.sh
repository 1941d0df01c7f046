# Round 2, call U: bench.py for the column and block splits at N = 1, and at N = 2 with both
# ranks on GPU 0 (exact sections and exact configs included), default steps trimmed.
set -o pipefail
mkdir -p gpurun_out/r02u
O=gpurun_out/r02u
for alg in colwise blockwise; do
  timeout -k 10 400 python bench.py --alg $alg --steps 50 --no-cpu-baseline > $O/n1_$alg.json 2> $O/n1_$alg.err || { tail -20 $O/n1_$alg.err; exit 1; }
  python -c "import json; d=json.load(open('$O/n1_$alg.json')); print('$alg', d['value'], d['roofline']['frac'], d['exact']['value'], d['exact']['kernel'])"
  MVG_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2955${#alg} bench.py --gpus 2 --alg $alg --steps 20 --e2e-iters 1 --config-steps 4 > $O/n2_$alg.json 2> $O/n2_$alg.err || { tail -30 $O/n2_$alg.err; exit 1; }
  python -c "import json; d=json.load(open('$O/n2_$alg.json')); print('$alg n2', d['value'], d['exact']['max_rel_vs_tree'], [c['exact']['max_rel_vs_tree'] for c in d['configs']])"
done
echo all-done
