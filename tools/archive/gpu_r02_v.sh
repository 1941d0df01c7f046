# Round 2, call V: the register forms with the chain hopping across lanes (gemv_seq_hop):
# exact-mode parity tests over every variant, then the sweep on the few-row and mid shapes.
set -o pipefail
mkdir -p gpurun_out/r02v
O=gpurun_out/r02v
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -2 $O/pytest_exact.log
timeout -k 10 600 python -u tools/sweep_exact.py 3 asym_1200x60000,asym_120x60000,ref_600sq,ref_1800sq,ref_4200sq,ref_10200sq,mid_4096x16384,mid_8192x16384,mid_8192x8192,mid_12288x12288,cfg2_16384sq,cfg3_g8_strip_65536x8192,cfg5_shard_524288x512 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
