# Round 2, call BG: read-rate calibration (tools/read_calibration.py: the tree GEMV beside
# address-order and per-range read-only kernels over the same bytes), then a short bench run
# to check the GFLOP/s fields.
set -o pipefail
mkdir -p gpurun_out/r02bg
O=gpurun_out/r02bg
timeout -k 10 300 python -u tools/read_calibration.py 7 16384,16384 65536,32768 524288,512 > $O/calib.jsonl 2> $O/calib.err || { tail -20 $O/calib.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline --steps 20 > $O/bench_short.json 2> $O/bench_short.err || { tail -20 $O/bench_short.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_short.json')); print(d['value'], d['gflops'], d['exact']['gflops'], d['end_to_end']['shared'])"
echo all-done
