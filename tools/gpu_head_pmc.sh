#!/bin/bash
# Counter passes over the SAM head alone (tools/head_bench.py, product form or
# SAMNERF_HEAD_V=<form> of the diagnostic build): instruction cache, instruction
# mix, waits.  usage (GPU box): bash tools/gpu_head_pmc.sh [form]
set -o pipefail
OUT="$GRAFT_REPO_ROOT/gpurun_out/headpmc${1:+_v$1}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
[ -n "$1" ] && export SAMNERF_HEAD_V=$1
VAR=${1:+--variants $1}
i=0
for set in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o p -- \
    python3 "$GRAFT_REPO_ROOT/tools/head_bench.py" $VAR --iters 3 --no-exact > "$OUT/p$i.log" 2>&1; rc=$?
  echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_table.py" "$OUT" | grep -i "sam_head\|kernel" | cut -c1-900
