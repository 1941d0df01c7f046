#!/usr/bin/env bash
# rocprofv3 counter passes over the exact GEMV (and the tree GEMV launched beside it) on one
# device-resident shape, one pass per counter group (rocprofv3 does not split groups over passes),
# each pass under its own hard time limit. Development tool (MI355X box).
#   tools/pmc_passes.sh OUTDIR M K VARIANT [VARIANT ...]
# VARIANT: an mvg_gemv_exact_variant_name, "auto" or "panels" (tools/exact_probe.py), or with
# PMC_PROBE=tools/multi_probe.py a vector count "nv<N>" (mvg_gemv_multi). Each pass lands in
# OUTDIR/<variant>/<group>/; summarise with tools/pmc_traffic.py.
set -euo pipefail
OUT="$1"; M="$2"; K="$3"; shift 3
PROBE="${PMC_PROBE:-tools/exact_probe.py}"
PASSES=(
  "fetch:FETCH_SIZE"
  "write:WRITE_SIZE"
  "l2:TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
  "ta:TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "sq:SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
)
for v in "$@"; do
  for g in "${PASSES[@]}"; do
    name="${g%%:*}"; counters="${g#*:}"
    mkdir -p "$OUT/$v/$name"
    # shellcheck disable=SC2086
    timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d "$OUT/$v/$name" \
        -- python3 "$PROBE" "$M" "$K" 10 "$v" > "$OUT/$v/$name/run.log" 2>&1
    echo "pmc $v $name done"
  done
done
