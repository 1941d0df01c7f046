# rocprofv3 PMC passes over the default bench (one counter group per pass, no tracing domains
# combined with --pmc). Usage: bash tools/gpu_pmc.sh [extra bench args]
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-configs --steps 10 --warmup 2 $*"
timeout -k 10 240 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU" "VALUBusy" "VALUUtilization" "MemUnitStalled" "SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE TA_BUSY_avr"; do
  tag=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  echo "== pmc $pass"
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $R/gpurun_out/pmc_$tag -o run -- $BENCH > $R/gpurun_out/pmc_$tag.log 2>&1 || { tail -5 $R/gpurun_out/pmc_$tag.log; exit 1; }
done
echo pmc-done
