#!/bin/bash
# PMC passes of bench.py for each value in $MODES of the variable $MODE_VAR
# (default SAMNERF_LOOKUP; one rocprofv3 --pmc run per counter group, counters
# only), then per-kernel tables.  PMC_GROUPS="..|.." replaces the counter groups.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmcab"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
  "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
  ${EXTRA_GROUP:+"$EXTRA_GROUP"}
)
if [ -n "${PMC_GROUPS:-}" ]; then IFS="|" read -r -a GROUPS_ <<< "$PMC_GROUPS"; fi
VAR=${MODE_VAR:-SAMNERF_LOOKUP}
for m in ${MODES:-packed box}; do
  i=0
  for g in "${GROUPS_[@]}"; do
    export "$VAR=$m"
    timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/$m/p$i" -o p$i \
      -- python "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --cpu-rays 0 --ref-gpu-rays 0 ${BENCH_ARGS:-} > "$OUT/${m}_p$i.log" 2>&1
    rc=$?; echo "$m pass $i rc=$rc"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
    i=$((i+1))
  done
  echo "== $m"; python "$GRAFT_REPO_ROOT/tools/pmc_table.py" "$OUT/$m" | grep -E "${KFILTER:-k_sgrid|k_prop_sigma|k_final}"
done
