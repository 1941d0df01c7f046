# PMC passes (tools/pmc_passes.sh) over the four dominant shapes: config 2, 5, 3 (G = 1), 4 (G = 1);
# development script, run through gpurun from the repo root; summarise with tools/pmc_traffic.py.
export TMPDIR=/tmp
OUT=gpurun_out/r4c; mkdir -p $OUT/pmc; for d in cfg2 cfg5 cfg3 cfg4; do mkdir -p $OUT/pmc/$d; cp profiles/r04/rocprofv3_counters_gfx950.txt $OUT/pmc/$d/; done
G="fetch write l2 valu mall tlb sq"
PMC_GROUPS="$G" bash tools/pmc_passes.sh $OUT/pmc/cfg2 16384 16384 auto panels > $OUT/p2.log 2>&1 || exit 1
PMC_GROUPS="$G" bash tools/pmc_passes.sh $OUT/pmc/cfg5 4194304 512 auto > $OUT/p5.log 2>&1 || exit 1
PMC_GROUPS="$G" bash tools/pmc_passes.sh $OUT/pmc/cfg3 65536 65536 auto > $OUT/p3.log 2>&1 || exit 1
PMC_GROUPS="$G" bash tools/pmc_passes.sh $OUT/pmc/cfg4 131072 131072 auto > $OUT/p4.log 2>&1 || exit 1
echo done
