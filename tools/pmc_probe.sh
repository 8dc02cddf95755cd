#!/bin/bash
# PMC probe: one rocprofv3 --pmc pass per counter group (counters only, no
# tracing domains), then a per-kernel table.  usage (on the GPU box):
#   bash tools/pmc_probe.sh [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
  "TCP_TCC_READ_REQ TCP_TOTAL_ACCESSES TCP_PENDING_STALL_CYCLES"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
)
i=0
for g in "${GROUPS_[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o p$i -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --cpu-rays 0 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($g) rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  i=$((i+1))
done
python "$GRAFT_REPO_ROOT/tools/pmc_table.py" "$OUT"
