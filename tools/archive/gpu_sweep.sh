# GPU parity tests, then a variant sweep: bash tools/gpu_sweep.sh <shapes> <variant prefixes> <out name>
set -o pipefail
mkdir -p gpurun_out
SHAPES=${1:-cfg2_16384sq}; PREFIX=${2:-rowblk}; OUT=${3:-sweep}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -u tools/sweep_variants.py 7 "$SHAPES" "$PREFIX" > gpurun_out/$OUT.jsonl 2> gpurun_out/$OUT.err || { tail gpurun_out/$OUT.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/$OUT.jsonl'):
    d=json.loads(l); print(d['shape'], d['variant'], d['median_us'], d['GBps_median'], d['GBps_best'], d['max_rel_vs_rocblas'])
"
