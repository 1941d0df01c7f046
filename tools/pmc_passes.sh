#!/usr/bin/env bash
# rocprofv3 counter passes over the exact GEMV (and the tree GEMV launched beside it) on one
# device-resident shape, one pass per counter group (rocprofv3 does not split groups over passes),
# each pass under its own hard time limit. Development tool (MI355X box).
#   tools/pmc_passes.sh OUTDIR M K VARIANT [VARIANT ...]
# VARIANT: an mvg_gemv_exact_variant_name, "auto" or "panels" (tools/exact_probe.py), or with
# PMC_PROBE=tools/multi_probe.py a vector count "nv<N>" (mvg_gemv_multi). Each pass lands in
# OUTDIR/<variant>/<group>/; summarise with tools/pmc_traffic.py. PMC_GROUPS="fetch valu ..."
# picks groups. A counter the box does not list (rocprofv3 -L, cached in OUTDIR/counters.txt) is
# dropped from its pass before the run: asking for an unknown counter fails the whole pass.
set -euo pipefail
OUT="$1"; M="$2"; K="$3"; shift 3
PROBE="${PMC_PROBE:-tools/exact_probe.py}"
mkdir -p "$OUT"
if [ ! -s "$OUT/counters.txt" ]; then
  timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
fi
PASSES=(
  "fetch:FETCH_SIZE"
  "write:WRITE_SIZE"
  "l2:TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
  "ta:TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "sq:SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
  # VALU busy (north_star's counter): SQ_ACTIVE_INST_VALU quad-cycles x 4 over SIMD-cycles
  "valu:SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "f64:SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  # memory-side requests: all of them, those that went to DRAM (the rest hit the MALL /
  # Infinity Cache), and the ones stalled for credits
  "ea:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RD_UNCACHED_32B_sum"
  "mall:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"
  # address translation in the L1 (UTCL1) and the vector-memory issue side
  "tlb:TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum"
  "tlb2:TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
  "vmem:SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  "tcp:TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
)
have() { grep -q -w -- "${1%_sum}" "$OUT/counters.txt"; }
for v in "$@"; do
  for g in "${PASSES[@]}"; do
    name="${g%%:*}"; counters="${g#*:}"
    if [ -n "${PMC_GROUPS:-}" ] && ! [[ " $PMC_GROUPS " == *" $name "* ]]; then continue; fi
    keep=""
    for c in $counters; do
      if have "$c"; then keep="$keep $c"; else echo "pmc $v $name: $c not listed on this box, dropped"; fi
    done
    [ -n "$keep" ] || continue
    mkdir -p "$OUT/$v/$name"
    # shellcheck disable=SC2086
    timeout -s KILL 90 rocprofv3 --pmc $keep --output-format csv -d "$OUT/$v/$name" \
        -- python3 "$PROBE" "$M" "$K" 10 "$v" > "$OUT/$v/$name/run.log" 2>&1
    echo "pmc $v $name done:$keep"
  done
done
