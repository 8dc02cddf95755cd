#!/bin/bash
# GPU-box check of the SAM-head forms (diagnostic build switch SAMNERF_HEAD_V):
# timing + bit identity (tools/head_bench.py), a kernel trace and one counter
# pass per form.  Every GPU step has its own time limit; a failure stops it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/head"
mkdir -p "$OUT"
V=${HEAD_VARIANTS:-1,2,3}
timeout -k 10 300 python tools/head_bench.py --variants "$V" > "$OUT/head.json" 2> "$OUT/head.err"; rc=$?
echo "head_bench rc=$rc"; cat "$OUT/head.json"; [ $rc -ne 0 ] && { tail -20 "$OUT/head.err"; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
  python3 "$GRAFT_REPO_ROOT/tools/head_bench.py" --variants "$V" --iters 5 --no-exact > "$OUT/trace.log" 2>&1; rc=$?
echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/trace.log"; exit $rc; }
grep -h "sam_head" "$OUT"/trace/*kernel_stats.csv | cut -d, -f1-4
for v in ${V//,/ }; do
  SAMNERF_HEAD_V=$v timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/pmc_v$v" -o p -- python3 "$GRAFT_REPO_ROOT/tools/head_bench.py" --variants "$v" --iters 3 --no-exact > "$OUT/pmc_v$v.log" 2>&1; rc=$?
  echo "pmc v$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/pmc_v$v.log"; exit $rc; }
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_table.py" "$OUT" | grep sam_head | cut -c1-600
