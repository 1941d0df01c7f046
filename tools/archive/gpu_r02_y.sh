# Round 2, call Y: chain-hopping forms with the waves per CU capped (dynamic LDS) on the tall
# shapes, where every wave of the grid is resident at once without the cap.
set -o pipefail
mkdir -p gpurun_out/r02y
O=gpurun_out/r02y
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
timeout -k 10 600 python -u tools/sweep_exact.py 3 cfg2_16384sq,mid_32768x16384,cfg3_g1_65536sq,tall_131072x16384,cfg4_block_65536x32768,mid_12288x12288 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
