# Round 2, call AM: the golden replay through the executables and the default bench on the
# final exact dispatch.
set -o pipefail
mkdir -p gpurun_out/r02am
O=gpurun_out/r02am
timeout -k 10 400 python -u tools/exact_golden_sweep.py > $O/golden_replay.jsonl 2> $O/golden_replay.err || { tail -20 $O/golden_replay.err; exit 1; }
tail -1 $O/golden_replay.jsonl
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['exact'], [(c['value'], c['exact']['value'], c['exact']['kernel']) for c in d['configs']], d['cpu_baseline']['value'])"
echo all-done
