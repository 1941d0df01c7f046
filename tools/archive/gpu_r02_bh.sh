# Round 2, call BH: panel copy allocated at first use — the full GPU suite and a short bench.
set -o pipefail
mkdir -p gpurun_out/r02bh
O=gpurun_out/r02bh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --no-configs --no-e2e --steps 50 > $O/bench_short.json 2> $O/bench_short.err || { tail -20 $O/bench_short.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_short.json')); print(d['value'], d['exact']['value'], d['exact']['kernel'], d['exact']['bit_identical_to_port'])"
echo all-done
