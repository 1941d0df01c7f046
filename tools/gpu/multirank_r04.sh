# Round-4: the driver's N-GPU bench command without a launcher, rehearsed with every rank on the
# one GPU of this box (MVG_SAME_DEVICE=1: RCCL over loopback sockets; times mean nothing, the
# N > 1 path runs end to end): N = 2 and N = 8. Output in gpurun_out/$OUT.
set -o pipefail
OUT=gpurun_out/${OUT:-m4a}
mkdir -p $OUT
for N in ${NS:-2 8}; do
  echo "== bench --gpus $N (no launcher, same device)"
  MVG_SAME_DEVICE=1 timeout -k 20 900 python bench.py --gpus $N --steps 20 --warmup 5 > $OUT/bench_n$N.json 2> $OUT/bench_n$N.err
  rc=$?; echo "rc=$rc"; tail -c 300 $OUT/bench_n$N.json; [ $rc -eq 0 ] || exit $rc
done
