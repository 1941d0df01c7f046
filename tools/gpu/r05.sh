# Round-5 check on one MI355X (gpurun, repo root). Steps chosen by STEPS (default
# "probe tests smoke bench"); output in gpurun_out/$OUT. Every GPU step runs under its own time
# limit; a test failure (rc 1) lets the later steps run, anything else (a fault, an abort, a
# time limit) ends the script there.
set -o pipefail
OUT=gpurun_out/${OUT:-r5a}
STEPS=${STEPS:-"probe tests smoke bench"}
TESTS=${TESTS:-tests}
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for step in $STEPS; do
  case $step in
  probe)
    echo "== lds refusal probe"
    timeout -k 10 60 ./tools/probes/lds_refusal > $OUT/lds_refusal.txt 2>&1; rc=$?
    cat $OUT/lds_refusal.txt; [ $rc -eq 0 ] || exit $rc
    (grep -E "MemTotal|MemAvailable" /proc/meminfo; cat /sys/fs/cgroup/memory.max /sys/fs/cgroup/memory.current;
     df -B1 /dev/shm; for i in /sys/devices/system/cpu/cpu0/cache/index*; do echo $i $(cat $i/level $i/type $i/size $i/shared_cpu_list); done;
     nproc; cat /sys/fs/cgroup/cpu.max; lscpu | grep -iE "model name|socket|L3|NUMA node") > $OUT/host.txt 2>&1
    cat $OUT/host.txt ;;
  tests)
    echo "== pytest gpu ($TESTS)"
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
    rc=$?; tail -5 $OUT/pytest_gpu.log; ok $rc || exit $rc ;;
  smoke)
    echo "== smoke"
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
    tail -2 $OUT/smoke.log; ok $rc || exit $rc ;;
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
  pmc)
    echo "== PMC passes at config 2: the evenly placed exact form (the bench's row-major exact kernel) + the tree kernel beside it"
    mkdir -p $OUT/pmc/cfg2
    PMC_GROUPS="fetch write l2 valu mall tlb" timeout -k 10 900 bash tools/pmc_passes.sh $OUT/pmc/cfg2 16384 16384 hop8e_l8_w2_u16_n8 \
        > $OUT/pmc_cfg2.log 2>&1; rc=$?
    tail -3 $OUT/pmc_cfg2.log; [ $rc -eq 0 ] || exit $rc
    python3 tools/pmc_traffic.py --outdir $OUT/pmc_summary --M 16384 --K 16384 $OUT/pmc/cfg2 ;;
  evprobe)
    echo "== event timing probe (untraced, then under the kernel trace)"
    timeout -k 10 120 python3 tools/probes/event_timing_probe.py 16384 16384 50 > $OUT/event_probe.jsonl 2> $OUT/event_probe.err; rc=$?
    cat $OUT/event_probe.jsonl; [ $rc -eq 0 ] || exit $rc
    cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/evprof -o run -- \
        python3 $ROOT/tools/probes/event_timing_probe.py 16384 16384 50 > $ROOT/$OUT/event_probe_traced.jsonl 2>> $ROOT/$OUT/event_probe.err; rc=$?
    cd $ROOT; cat $OUT/event_probe_traced.jsonl; [ $rc -eq 0 ] || exit $rc ;;
  torchprobe)
    echo "== PyTorch's own HIP runtime beside the library's: which orders work, and the tree kernel's time in each"
    for mode in ${TORCH_MODES:-none set late sync none late}; do
      timeout -k 10 120 python3 tools/probes/event_timing_probe.py 16384 16384 100 tree $mode >> $OUT/torch_probe.jsonl 2>> $OUT/torch_probe.err
      rc=$?; echo "mode $mode rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
    done
    cat $OUT/torch_probe.jsonl ;;
  streamprobe)
    echo "== tree kernel per stream, 4 processes"
    for i in 1 2 3 4; do
      timeout -k 10 120 python3 tools/probes/stream_probe.py 16384 16384 6 100 >> $OUT/stream_probe.jsonl 2>> $OUT/stream_probe.err || exit $?
    done
    cat $OUT/stream_probe.jsonl ;;
  settle)
    echo "== headline only, fresh processes: no settle vs the settle before the W = 5 warm-up steps, interleaved"
    for i in 1 2 3 4 5 6; do for st in ${SETTLE:-1.5} 0; do
      timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --settle-s $st --no-exact --no-cpu-baseline --no-e2e \
          --no-configs --no-multi --no-loader >> $OUT/settle.jsonl 2>> $OUT/settle.err || exit $?
    done; done
    python3 -c "
import json
for l in open('$OUT/settle.jsonl'):
    d = json.loads(l); st = d.get('settle') or {}
    print(st.get('s'), st.get('first_us_per_step'), d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], st.get('trace_s_us', [])[:8])" ;;
  freshbox)
    echo "== the first GPU process of the call: config 2's kernel over the first minute"
    (rocm-smi --showmeminfo vram --showuse 2>&1 | tail -15) > $OUT/smi_before.txt
    timeout -k 10 100 python3 tools/probes/fresh_box_probe.py ${FRESH_S:-60} 16384 16384 ${FRESH_PAUSE:-0.5} > $OUT/fresh_box.jsonl 2> $OUT/fresh_box.err || exit $?
    ls /sys/bus/pci/devices/*/pp_dpm_sclk > $OUT/dpm_files.txt 2>&1 || true
    python3 -c "
import json
rows = [json.loads(l) for l in open('$OUT/fresh_box.jsonl')]
print([(r['t'], r['us']) for r in rows[:6]], '...', [(r['t'], r['us']) for r in rows[-3:]])" ;;
  gcorder)
    # bench_prev.py: `git show 4544303:bench.py > bench_prev.py` at the repo root for the run (not committed)
    echo "== headline only, interleaved: the collection after the settle (bench_prev.py) against before it (bench.py)"
    for i in 1 2 3 4 5 6; do for b in bench_prev.py bench.py; do
      timeout -k 10 120 python3 $b --steps 20 --warmup 5 --no-exact --no-cpu-baseline --no-e2e \
          --no-configs --no-multi --no-loader | sed "s/^{/{\"script\": \"$b\", /" >> $OUT/gcorder.jsonl 2>> $OUT/gcorder.err || exit $?
    done; done
    python3 -c "
import json
for l in open('$OUT/gcorder.jsonl'):
    d = json.loads(l); print(d['script'], d['value'], d['roofline']['kernel_ms'], d['ms_per_step'])" ;;
  idlegap)
    echo "== does an idle gap (sleep, gc.collect) before 20 launches change their per-launch times?"
    timeout -k 10 120 python3 tools/probes/idle_gap_probe.py ${GAP_ROUNDS:-4} > $OUT/idle_gap.jsonl 2> $OUT/idle_gap.err || exit $?
    python3 -c "
import json, collections
by = collections.defaultdict(list)
for l in open('$OUT/idle_gap.jsonl'):
    r = json.loads(l); by[str(r['gap'])].append(r)
for g, rs in by.items():
    print(g, [r['idle_ms'] for r in rs][:2], 'mean', [r['mean_us'] for r in rs], 'first5', [r['first5_us'] for r in rs], 'last5', [r['last5_us'] for r in rs], [r['sclk_after'] for r in rs][:2])" ;;
  evcost)
    echo "== headline only: does timing the kernel with HIP events slow the steps? span events vs none, interleaved"
    for i in 1 2 3 4 5 6; do for ev in -1 0; do
      timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --event-every $ev --no-exact --no-cpu-baseline --no-e2e \
          --no-configs --no-multi --no-loader >> $OUT/evcost.jsonl 2>> $OUT/evcost.err || exit $?
    done; done
    python3 -c "
import json
for l in open('$OUT/evcost.jsonl'):
    d = json.loads(l); print(d['roofline']['kernel_ms'], d['value'], d['ms_per_step'], (d.get('settle') or {}).get('last_us_per_step'))" ;;
  rehearse8)
    echo "== N=8 same-device rehearsal with a 120 s budget (the launcher-free form: bench.py starts the ranks)"
    MVG_SAME_DEVICE=1 timeout -k 30 400 python3 bench.py --gpus 8 --steps 5 --warmup 2 --budget-s 120 \
        > $OUT/bench_n8.json 2> $OUT/bench_n8.err; rc=$?
    tail -c 400 $OUT/bench_n8.json; grep "bench:" $OUT/bench_n8.err | tail -5; ok $rc || exit $rc ;;
  rehearse4)
    echo "== N=4 same-device rehearsal with the driver's defaults (budget 420 s): the whole line within the limit"
    MVG_SAME_DEVICE=1 timeout -k 30 600 python3 bench.py --gpus 4 --steps 20 --warmup 5 \
        > $OUT/bench_n4.json 2> $OUT/bench_n4.err; rc=$?
    tail -c 600 $OUT/bench_n4.json; grep "bench:" $OUT/bench_n4.err | tail -8; ok $rc || exit $rc ;;
  rehearse8d)
    echo "== N=8 same-device rehearsal with the driver's defaults (budget 420 s; loopback sockets: the worst case)"
    MVG_SAME_DEVICE=1 timeout -k 30 700 python3 bench.py --gpus 8 --steps 20 --warmup 5 \
        > $OUT/bench_n8d.json 2> $OUT/bench_n8d.err; rc=$?
    tail -c 600 $OUT/bench_n8d.json; grep "bench:" $OUT/bench_n8d.err | tail -8; ok $rc || exit $rc ;;
  sigterm8)
    echo "== N=8 same-device run terminated by a time limit mid-run: the line so far must come out (last step)"
    MVG_SAME_DEVICE=1 timeout -s TERM -k 60 75 python3 bench.py --gpus 8 --steps 5 --warmup 2 \
        > $OUT/bench_n8_sigterm.json 2> $OUT/bench_n8_sigterm.err; rc=$?
    echo "rc=$rc"; tail -c 600 $OUT/bench_n8_sigterm.json; grep "bench:" $OUT/bench_n8_sigterm.err | tail -5
    exit 0 ;;
  esac
done
