# The bench's one-process-per-GPU path at world size 1 under torch.distributed.run (RCCL process
# group, engine comm from the group, forced collectives, shared-memory + root-send distribution).
set -o pipefail
mkdir -p gpurun_out
for alg in rowwise colwise blockwise; do
MVG_BENCH_FORCE_DIST=1 MVG_ALWAYS_COLLECT=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --alg $alg --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/dist1_$alg.json 2> gpurun_out/dist1_$alg.err || { tail -30 gpurun_out/dist1_$alg.err; exit 1; }
cat gpurun_out/dist1_$alg.json
done
