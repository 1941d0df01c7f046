set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -k "numa or mpiexec or shared" -x -v --timeout 200 --timeout-method thread > gpurun_out/numa_apps.log 2>&1 || { tail -30 gpurun_out/numa_apps.log; exit 1; }
grep -cE "PASSED" gpurun_out/numa_apps.log; tail -1 gpurun_out/numa_apps.log
