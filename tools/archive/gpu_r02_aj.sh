# Round 2, call AJ: chain-hopping forms whose rows start their main segments on a 128-B line
# (masked head and tail segments) — exact tests, then the sweep over aligned, line-misaligned,
# odd-width and the reference's own shapes.
set -o pipefail
mkdir -p gpurun_out/r02aj
O=gpurun_out/r02aj
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1 || { tail -30 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
timeout -k 10 900 python -u tools/sweep_exact.py 3 cfg2_16384sq,even_16384x16386,even_16384x16388,odd_16384x16383,odd_65536x8191,odd_4096x16383,odd_1200x60001,odd_10200x1275,odd_4200x525,ref_4200sq,ref_10200sq,ref_1800sq,asym_1200x60000,asym_120x60000,mid_4096x16384,mid_8192x16384,mid_8192x8192,mid_12288x12288,mid_32768x16384,cfg3_g8_strip_65536x8192,cfg4_block_65536x32768,cfg5_shard_524288x512,cfg3_g1_65536sq,mid_2048x65536 > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
echo all-done
