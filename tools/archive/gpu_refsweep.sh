# GPU tests, small-size per-multiply costs, and the reference's test.sh sweep with the executables.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u tools/small_sizes.py rowwise > gpurun_out/small_rowwise.jsonl 2> gpurun_out/small.err || { tail gpurun_out/small.err; exit 1; }
cat gpurun_out/small_rowwise.jsonl
rm -rf gpurun_out/ref_sweep_g1
timeout -k 10 900 python tools/ref_sweep.py --out gpurun_out/ref_sweep_g1 > gpurun_out/ref_sweep.log 2>&1 || { tail gpurun_out/ref_sweep.log; exit 1; }
echo ref-sweep-done
