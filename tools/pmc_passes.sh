#!/bin/bash
# rocprofv3 PMC passes for the rooflines (one counter group per pass,
# counters only, no tracing domains).  usage (GPU box): [PASSES="i j"] bash tools/pmc_passes.sh TAG [bench args]
set -o pipefail
TAG=${1:-r2}; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
  "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "TA_BUSY_avr TA_BUSY_max SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE"
  "SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
)
# PASSES="4 5": only those groups (default: all)
i=0
for g in "${GROUPS_[@]}"; do
  if [ -n "${PASSES:-}" ] && ! [[ " $PASSES " == *" $i "* ]]; then i=$((i+1)); continue; fi
  timeout -s KILL 150 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o p$i -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --cpu-rays 0 --ref-gpu-rays 0 --no-alt --streams 1 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($g) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
  i=$((i+1))
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_table.py" "$OUT" > "$OUT/table.txt"
cat "$OUT/table.txt" | cut -c1-400
