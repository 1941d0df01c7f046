# Round 2, call X: the exact dispatch with the chain-hopping forms — full GPU suite, smoke,
# the final sweep of the exact variants, the golden replay through the executables, bench.
set -o pipefail
mkdir -p gpurun_out/r02x
O=gpurun_out/r02x
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 600 python -u tools/sweep_exact.py 3 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
timeout -k 10 400 python -u tools/exact_golden_sweep.py > $O/golden_replay.jsonl 2> $O/golden_replay.err || { tail -20 $O/golden_replay.err; exit 1; }
tail -1 $O/golden_replay.jsonl
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['exact']['value'], d['exact']['kernel'], [(c['value'], c['exact']['value']) for c in d['configs']])"
echo all-done
