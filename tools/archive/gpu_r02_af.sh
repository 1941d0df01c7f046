# Round 2, call AF: the tree dispatch with unaligned 16-B kernels for odd widths — parity tests,
# the odd-width sweep again (the dispatch's choice is `auto`), then the default bench.
set -o pipefail
mkdir -p gpurun_out/r02af
O=gpurun_out/r02af
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
timeout -k 10 600 python -u tools/sweep_variants.py 3 16384x16383,65536x8191,4096x16383,1200x60001,10200x1275,4200x525,524288x511,2048x65535,16384x16384 rowblk_w4_r2_u8_xcd$,scl_l64_r4_u4_nt1$,rowblk_w4_r2_u8$ > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['exact']['value'], [(c['value'], c['exact']['value']) for c in d['configs']])"
echo all-done
