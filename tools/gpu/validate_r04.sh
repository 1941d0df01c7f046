# Round-4 checks on one MI355X (gpurun, repo root): the exact kernel's pattern calibration on the
# same box, bench.py --gpus 2 started WITHOUT a launcher (both ranks on GPU 0), and the driver's
# N = 1 bench under rocprofv3's kernel trace. Output in gpurun_out/$OUT.
set -o pipefail
OUT=gpurun_out/${OUT:-v4a}
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
echo "== exact pattern calibration"
timeout -k 10 120 ./tools/micro/window_read 16384 16384 > $OUT/window_read.jsonl || exit $?
timeout -k 10 240 python -u tools/sweep_exact.py 5 cfg2_16384sq > $OUT/sweep_cfg2.jsonl 2> $OUT/sweep.err || exit $?
echo "== bench --gpus 2, no launcher, same device"
MVG_SAME_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_n2.json 2> $OUT/bench_n2.err
echo "rc=$?"; tail -c 300 $OUT/bench_n2.json
echo "== bench N=1 under rocprofv3"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o run -- \
    python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/bench.json 2> $ROOT/$OUT/bench.err || { tail $ROOT/$OUT/bench.err; exit 1; }
cd $ROOT && python3 tools/rocprof_by_grid.py $OUT/prof --out $OUT/kernel_by_grid.csv
tail -c 300 $OUT/bench.json
