# Round 2, call W: second sweep of the chain-hopping register forms (deeper pipelines, wider
# lane segments, more lanes per row) over few-row, mid and tall shapes, after the parity tests.
set -o pipefail
mkdir -p gpurun_out/r02w
O=gpurun_out/r02w
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -2 $O/pytest_exact.log
timeout -k 10 900 python -u tools/sweep_exact.py 3 asym_1200x60000,asym_120x60000,ref_600sq,ref_1800sq,ref_4200sq,ref_10200sq,mid_4096x16384,mid_8192x16384,mid_8192x8192,mid_12288x12288,cfg2_16384sq,mid_32768x16384,mid_2048x65536,mid_4096x32768,cfg3_g8_strip_65536x8192,cfg5_shard_524288x512,cfg4_block_65536x32768,tall_131072x16384 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
