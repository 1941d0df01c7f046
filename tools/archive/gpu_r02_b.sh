# Round 2, call B: the whole GPU suite on the DPP-epilogue build, smoke, then the driver's
# scaling command rehearsed at N = 8 with every rank on GPU 0 (RCCL over loopback sockets).
set -o pipefail
mkdir -p gpurun_out/r02b
O=gpurun_out/r02b
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== same-device N=8"
MVG_SAME_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29548 bench.py --gpus 8 > $O/same8.json 2> $O/same8.err || { tail -30 $O/same8.err; exit 1; }
python -c "import json; d=json.load(open('$O/same8.json')); print(8, d['value'], d['config']['R'], d['end_to_end'].get('roofline'), [c.get('config') for c in d['configs']])"
echo all-done
