# Round 2, call AK: the exact dispatch on line alignment (LDS forms only for line-aligned tall
# shapes, chain-hopping forms with 8-B loads elsewhere) — exact tests, the sweep over every
# shape, the default bench.
set -o pipefail
mkdir -p gpurun_out/r02ak
O=gpurun_out/r02ak
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
timeout -k 10 900 python -u tools/sweep_exact.py 3 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['exact']['value'], d['exact']['kernel'], [(c['value'], c['exact']['value'], c['exact']['kernel']) for c in d['configs']])"
echo all-done
