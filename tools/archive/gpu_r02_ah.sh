# Round 2, call AH: 8-B chain-hopping forms that peel a misaligned row's first column so its
# segment loads are 16-B aligned — exact tests, then the odd-width sweep.
set -o pipefail
mkdir -p gpurun_out/r02ah
O=gpurun_out/r02ah
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
timeout -k 10 700 python -u tools/sweep_exact.py 3 odd_4200x525,odd_10200x1275,odd_16384x16383,odd_1200x60001,odd_65536x8191,odd_4096x16383,cfg2_16384sq,asym_1200x60000 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
