set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03q
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "whole_y" --timeout 150 --timeout-method thread > gpurun_out/r03q/pytest_whole_y.log 2>&1
