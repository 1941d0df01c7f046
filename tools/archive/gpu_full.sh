# Full round refresh: tests, smoke, bench, rocprof, PMC (config 2), reference sweep, config sweep + PMC.
set -o pipefail
bash tools/gpu_round.sh || exit $?
for d in gpurun_out/pmc_*/; do n=$(basename $d); rm -rf gpurun_out/cfg2_$n; mv $d gpurun_out/cfg2_$n; done
timeout -k 10 900 python tools/ref_sweep.py --out gpurun_out/ref_sweep_g1 > gpurun_out/ref_sweep.log 2>&1 || { tail gpurun_out/ref_sweep.log; exit 1; }
echo ref-sweep-done
bash tools/gpu_configs.sh
