# Round 2, call G: the driver's exact bench command (python bench.py, defaults) under
# rocprofv3 --kernel-trace --stats, so the committed summary is of the same command; the trace is
# then grouped by launch grid (config 2 / exact / configs 3-5 share kernel names).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json | head -c 600; echo
cat $O/prof/run_kernel_stats.csv
python3 $R/tools/rocprof_by_grid.py $O/prof --out $O/by_grid.csv && cat $O/by_grid.csv
rm -f $O/prof/run_kernel_trace.csv.gz
echo all-done
