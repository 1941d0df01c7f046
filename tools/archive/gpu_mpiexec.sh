# The executables launched like the reference (mpiexec -n P), on one GPU: app tests, then the
# rank-mode path at P = 1 on config 2 (shared window vs root send) beside the single-process run.
set -o pipefail
mkdir -p gpurun_out/mpiexec/data/out
timeout -k 10 300 python -u -m pytest tests/test_apps.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/mpiexec/pytest_apps.log 2>&1 || { tail -30 gpurun_out/mpiexec/pytest_apps.log; exit 1; }
tail -3 gpurun_out/mpiexec/pytest_apps.log
cd gpurun_out/mpiexec
for mode in single shared send; do
  case $mode in
    single) cmd="../../bin/multiplier_rowwise 16384 16384"; extra="";;
    shared) cmd="/opt/conda/bin/mpiexec -n 1 ../../bin/multiplier_rowwise 16384 16384"; extra="MVG_RANK_MODE=1 MVG_ALWAYS_COLLECT=1";;
    send) cmd="/opt/conda/bin/mpiexec -n 1 ../../bin/multiplier_rowwise 16384 16384"; extra="MVG_RANK_MODE=1 MVG_ALWAYS_COLLECT=1 MVG_DIST=send";;
  esac
  env $extra MVG_SYNTH=1 MVG_ITERS=20 timeout -k 10 200 $cmd > run_$mode.txt 2>&1 || { tail -20 run_$mode.txt; exit 1; }
  echo "== $mode"; grep -E "end-to-end|device-resident|launch:" run_$mode.txt
done
