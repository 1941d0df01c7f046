# Round 2, call Z: PMC passes (FETCH_SIZE; WRITE_SIZE — separate runs) over the chain-hopping
# exact kernels at their dispatch shapes, then the driver's bench command under a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for shape in "8192 16384" "1200 60000" "65536 65536"; do
  tag=$(echo $shape | tr ' ' x)
  for pass in FETCH_SIZE WRITE_SIZE; do
    ptag=$(echo $pass | tr 'A-Z' 'a-z')
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $O/${tag}_$ptag -o run -- python3 $R/tools/exact_probe.py $shape 8 > $O/${tag}_$ptag.log 2>&1 || { tail -5 $O/${tag}_$ptag.log; exit 1; }
  done
done
cd $R
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_trace -o run -- python3 bench.py > $O/bench_trace.json 2> $O/bench_trace.err || { tail -20 $O/bench_trace.err; exit 1; }
echo all-done
