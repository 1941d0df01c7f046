# A/B of the exchange placement at world size 1 with forced collectives (rowwise, config 2).
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" MVG_ALWAYS_COLLECT=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 100 > gpurun_out/ab_$name.json 2>> gpurun_out/ab.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
run serial MVG_XRING=1
run ring8_nofence MVG_XRING=8
run ring8_timing MVG_XRING=8 MVG_XEV=0
run ring8_timing_nofence MVG_XRING=8 MVG_XEV=0x20000000
run ring8_dev MVG_XRING=8 MVG_XEV=0x40000002
done
R=$PWD; cd /tmp && export TMPDIR=/tmp
MVG_XEV=0 MVG_ALWAYS_COLLECT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_x -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 2 > /dev/null 2>> $R/gpurun_out/ab.err || exit 1
