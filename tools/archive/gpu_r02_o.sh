# Round 2, call O: default bench (reference baseline on two placements), then the reference's
# test.sh sizes with the executables in bit-exact mode.
set -o pipefail
mkdir -p gpurun_out/r02o
O=gpurun_out/r02o
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); c=d['cpu_baseline']; print(d['value'], d['roofline']['frac'], c['value'], c['placement'], c['port']['value'])"
rm -rf $O/ref_sweep_exact
MVG_EXACT=1 timeout -k 10 900 python tools/ref_sweep.py --out $O/ref_sweep_exact > $O/ref_sweep.log 2>&1 || { tail $O/ref_sweep.log; exit 1; }
echo all-done
