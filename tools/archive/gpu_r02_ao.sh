# Round 2, call AO: shallower 8-lane chain-hopping forms (fewer VGPRs, more waves resident) on
# the tall shapes where the grid needs several rounds of waves, after the exact tests.
set -o pipefail
mkdir -p gpurun_out/r02ao
O=gpurun_out/r02ao
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
timeout -k 10 700 python -u tools/sweep_exact.py 3 cfg3_g8_strip_65536x8192,cfg4_block_65536x32768,tall_131072x16384,tall_262144x8192,mid_32768x16384,cfg2_16384sq,cfg5_shard_524288x512,cfg3_g1_65536sq,mid_12288x12288 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
