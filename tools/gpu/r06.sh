# Round-6 runs on one MI355X (gpurun, repo root). Steps chosen by STEPS; output in
# gpurun_out/$OUT. Every GPU step runs under its own time limit; a test failure (rc 1) lets the
# later steps run, anything else (a fault, an abort, a time limit) ends the script there.
set -o pipefail
OUT=gpurun_out/${OUT:-r6a}
STEPS=${STEPS:-"host smoke"}
TESTS=${TESTS:-tests}
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for step in $STEPS; do
  case $step in
  host)
    (grep -E "MemTotal|MemAvailable" /proc/meminfo; cat /sys/fs/cgroup/memory.max /sys/fs/cgroup/memory.current;
     df -B1 /dev/shm; nproc; cat /sys/fs/cgroup/cpu.max; lscpu | grep -iE "model name|socket|NUMA node";
     for f in /sys/kernel/mm/transparent_hugepage/shmem_enabled /sys/kernel/mm/transparent_hugepage/enabled \
              /sys/kernel/mm/transparent_hugepage/defrag /proc/sys/vm/nr_hugepages; do echo "$f: $(cat $f)"; done;
     uname -r) > $OUT/host.txt 2>&1
    cat $OUT/host.txt ;;
  hostprobe)
    echo "== host matrix setup: fill and page-lock timed apart (anon / shm / shm_falloc; P processes x T threads)"
    timeout -k 10 ${HP_LIMIT:-400} python3 tools/probes/host_setup_probe.py ${HP_GIB:-32} ${HP_MODES:-anon,shm,shm_falloc} \
        ${HP_P:-1,4} ${HP_T:-16,4} > $OUT/host_setup.jsonl 2> $OUT/host_setup.err; rc=$?
    python3 -c "
import json
for l in open('$OUT/host_setup.jsonl'):
    d = json.loads(l)
    if 'host' in d: print(d); continue
    print(d['mode'], 'P', d['P'], 'T', d['T'], 'fill', d['fill_GBps'], 'pin', d['pin_GBps'], 'setup', d.get('setup_GBps'), 'GB/s; wall', d['wall_s'],
          [(r['alloc_s'], r['fill_s'], r['pin_s'], r.get('unpin_s')) for r in d['per_process']][:4])"
    [ $rc -eq 0 ] || { tail $OUT/host_setup.err; exit $rc; } ;;
  smoke)
    echo "== smoke"
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
    tail -3 $OUT/smoke.log; ok $rc || exit $rc ;;
  tests)
    echo "== pytest gpu ($TESTS)"
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
    rc=$?; tail -5 $OUT/pytest_gpu.log; ok $rc || exit $rc ;;
  pmc3)
    # the tree kernel (gemv_rowblock<4,2,8>) on config 2's shard, config 4 on one GPU and config
    # 4's per-GPU block of the 2 x 4 grid, same box: reads in flight, read latency, translation
    echo "== PMC passes, tree kernel alone, three shapes"
    for shape in "16384 16384" "131072 131072" "65536 32768"; do
      set -- $shape; d=$OUT/pmc/tree_$1x$2
      mkdir -p $d
      PMC_GROUPS="${PMC_GROUPS:-fetch write valu mall tlb tlb2 tcp}" timeout -k 10 600 bash tools/pmc_passes.sh $d $1 $2 tree \
          > $OUT/pmc_$1x$2.log 2>&1; rc=$?
      tail -2 $OUT/pmc_$1x$2.log; [ $rc -eq 0 ] || exit $rc
      python3 tools/pmc_traffic.py --outdir $OUT/pmc_summary --M $1 --K $2 $d || exit $?
    done ;;
  shapes)
    # the tree kernel alone, 50 launches per shape, under the kernel trace: config 2's shard,
    # config 4 on one GPU, config 4's per-GPU block of the 2 x 4 grid
    echo "== tree kernel durations, three shapes"
    for shape in "16384 16384" "131072 131072" "65536 32768"; do
      set -- $shape
      sleep ${SHAPES_GAP:-0}  # let the driver finish clearing the previous process's VRAM
      cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/shapes/$1x$2 -o run -- \
          python3 $ROOT/tools/exact_probe.py $1 $2 50 tree > $ROOT/$OUT/shapes_$1x$2.log 2>&1; rc=$?
      cd $ROOT; [ $rc -eq 0 ] || { tail $OUT/shapes_$1x$2.log; exit $rc; }
      python3 tools/rocprof_by_grid.py $OUT/shapes/$1x$2 --out $OUT/shapes/kernel_by_grid_$1x$2.csv || exit $?
      head -3 $OUT/shapes/kernel_by_grid_$1x$2.csv
    done ;;
  sliceprobe)
    echo "== config 4's single-GPU launch: whole, split, and slice by slice, beside config 2's shape"
    timeout -k 10 180 python3 tools/probes/slice_probe.py --rounds ${SP_ROUNDS:-4} --pre-gib "${SP_PRE:-}" > $OUT/slice_probe.jsonl 2> $OUT/slice_probe.err; rc=$?
    cat $OUT/slice_probe.jsonl; [ $rc -eq 0 ] || { tail $OUT/slice_probe.err; exit $rc; } ;;
  bench2)
    echo "== bench N=1 twice back to back, no CPU sections (the second starts while the first's VRAM is being cleared)"
    for i in 1 2; do
      timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-multi --no-loader \
          > $OUT/bench2_$i.json 2> $OUT/bench2_$i.err; rc=$?; ok $rc || exit $rc
      python3 -c "
import json
p = json.loads(open('$OUT/bench2_$i.json').read().strip().splitlines()[-1])
print($i, p['value'], p['roofline']['frac'], p.get('vram_wait'), [(c['config'], c.get('kernel_frac'), c.get('vram_wait')) for c in p['configs']])"
    done ;;
  bench)
    echo "== bench N=1 (the driver's command)"
    timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; rc=$?
    tail -c 300 $OUT/bench.json; tail -3 $OUT/bench.err; ok $rc || exit $rc ;;
  benchprof)
    echo "== bench N=1 under rocprofv3 --kernel-trace --stats"
    cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o run -- \
        python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/bench_prof.json 2> $ROOT/$OUT/bench_prof.err; rc=$?
    cd $ROOT; ok $rc || { tail $OUT/bench_prof.err; exit $rc; }
    python3 tools/rocprof_by_grid.py $OUT/prof --out $OUT/kernel_by_grid.csv ;;
  rehearse4)
    echo "== N=4 same-device rehearsal with the driver's defaults (budget 420 s)"
    MVG_SAME_DEVICE=1 timeout -k 30 600 python3 bench.py --gpus 4 --steps 20 --warmup 5 \
        > $OUT/bench_n4.json 2> $OUT/bench_n4.err; rc=$?
    tail -c 600 $OUT/bench_n4.json; grep "bench:" $OUT/bench_n4.err | tail -8; ok $rc || exit $rc ;;
  rehearse2l)
    echo "== N=2 same-device rehearsal, the driver's own launcher command, default budget"
    MVG_SAME_DEVICE=1 timeout -k 30 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
        > $OUT/bench_n2.json 2> $OUT/bench_n2.err; rc=$?
    tail -c 600 $OUT/bench_n2.json; grep "bench:" $OUT/bench_n2.err | tail -8; ok $rc || exit $rc ;;
  rehearse8d)
    echo "== N=8 same-device rehearsal with the driver's defaults (budget 420 s; loopback sockets: the worst case)"
    MVG_SAME_DEVICE=1 timeout -k 30 700 python3 bench.py --gpus 8 --steps 20 --warmup 5 \
        > $OUT/bench_n8d.json 2> $OUT/bench_n8d.err; rc=$?
    tail -c 600 $OUT/bench_n8d.json; grep "bench:" $OUT/bench_n8d.err | tail -8; ok $rc || exit $rc ;;
  esac
done
