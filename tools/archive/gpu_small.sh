# Small-size per-multiply costs (host wall, enqueue, kernel events) + a kernel trace of one pass.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/small_sizes.py rowwise > gpurun_out/small_rowwise.jsonl 2> gpurun_out/small.err || { tail gpurun_out/small.err; exit 1; }
cat gpurun_out/small_rowwise.jsonl
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_small -o run --output-format csv -- python3 $R/tools/small_sizes.py rowwise > /dev/null 2>> $R/gpurun_out/small.err || exit 1
cd $R && cat gpurun_out/prof_small/run_kernel_stats.csv
