# bench.py's configs 3-5 section: N = 1 on the GPU, then the driver's N = 2 and N = 8 commands
# with every rank on GPU 0 (MVG_SAME_DEVICE=1; timings of N > 1 mean nothing there).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/cb1.json 2> gpurun_out/cb1.err || { tail -30 gpurun_out/cb1.err; exit 1; }
echo "wall $SECONDS s"
python -c "import json; d=json.load(open('gpurun_out/cb1.json')); print(d['value'], d['roofline']['frac']); [print(c) for c in d['configs']]"
timeout -k 10 300 python -u -m pytest tests/test_apps.py -k bench_two_ranks -x -v --timeout 200 --timeout-method thread > gpurun_out/cb_test.log 2>&1 || { tail -30 gpurun_out/cb_test.log; exit 1; }
tail -2 gpurun_out/cb_test.log
MVG_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29548 bench.py --gpus 8 > gpurun_out/cb8.json 2> gpurun_out/cb8.err || { tail -30 gpurun_out/cb8.err; exit 1; }
echo "wall $SECONDS s"
python -c "import json; d=json.load(open('gpurun_out/cb8.json')); print(d['value']); [print(c) for c in d['configs']]"
