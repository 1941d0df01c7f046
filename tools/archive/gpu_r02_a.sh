# Round 2, call A: DPP-reduction variants (parity, then a short-row sweep), the bench with the
# PCIe roofline, the bench's GEMV under rocprofv3 --kernel-trace --stats, and HBM PMC passes.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r02a
O=$R/gpurun_out/r02a
echo "== parity (all variants)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "all_variants or padded_lda or full_size" > $O/pytest_variants.log 2>&1 || { tail -20 $O/pytest_variants.log; exit 1; }
tail -2 $O/pytest_variants.log
echo "== sweep short rows"
timeout -k 10 400 python -u tools/sweep_variants.py 5 \
  cfg5_full_4194304x512,cfg5_shard_524288x512,mid_2097152x1024,mid_1048576x2048,mid_524288x4096,ref_1800sq,ref_4200sq,ref_10200sq vec \
  > $O/sweep_dpp.jsonl 2> $O/sweep_dpp.err || { tail -20 $O/sweep_dpp.err; exit 1; }
echo "== bench"
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-configs --steps 200 --warmup 20"
echo "== rocprofv3 stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- $BENCH > $O/prof_stats.json 2> $O/prof_stats.err || { tail -20 $O/prof_stats.err; exit 1; }
cat $O/prof_stats.json
for pass in FETCH_SIZE WRITE_SIZE; do
  tag=$(echo $pass | tr 'A-Z' 'a-z')
  echo "== pmc $pass"
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $O/pmc_$tag -o run -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-configs --steps 10 --warmup 2 > $O/pmc_$tag.log 2>&1 || { tail -5 $O/pmc_$tag.log; exit 1; }
done
echo all-done
