# All BASELINE configs on this box's GPU(s) + PMC passes for the non-default ones.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/configs.jsonl
timeout -k 10 900 python tools/config_sweep.py --out gpurun_out/configs.jsonl || exit $?
bash tools/gpu_pmc.sh --alg colwise --rows 65536 --cols 65536 > gpurun_out/pmc_cfg3.log 2>&1 || { tail gpurun_out/pmc_cfg3.log; exit 1; }
for d in fetch_size write_size tcc_hit_sum sq_waves; do rm -rf gpurun_out/cfg3_pmc_$d; mv gpurun_out/pmc_$d gpurun_out/cfg3_pmc_$d; done
bash tools/gpu_pmc.sh --alg rowwise --rows 4194304 --cols 512 > gpurun_out/pmc_cfg5.log 2>&1 || { tail gpurun_out/pmc_cfg5.log; exit 1; }
for d in fetch_size write_size tcc_hit_sum sq_waves; do rm -rf gpurun_out/cfg5_pmc_$d; mv gpurun_out/pmc_$d gpurun_out/cfg5_pmc_$d; done
echo configs-done
