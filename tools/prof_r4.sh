#!/bin/bash
# Round-4 measurement set (GPU box): the VALU issue-rate microbenchmark and its
# PMC pass, a headline-only kernel trace (bench.py --no-alt, one stream), and
# the PMC passes of the view (tools/pmc_passes.sh, incl. the wait-state group).
# Every step has its own time limit; a failure ends the script.
set -o pipefail
TAG=${1:-r4}
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 tools/bin/valu_rate > "$OUT/valu_rate.json" 2> "$OUT/valu_rate.err" || { echo "valu_rate failed"; exit 1; }
cat "$OUT/valu_rate.json"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/valu_pmc" -o v -- "$GRAFT_REPO_ROOT/tools/bin/valu_rate" 1024 > "$OUT/valu_pmc.log" 2>&1 || { echo "valu pmc failed"; tail -5 "$OUT/valu_pmc.log"; exit 1; }
echo "valu pmc ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --no-alt --streams 1 --steps 20 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log" | cut -c1-300
echo "trace ok"
if [ "${SKIP_PMC:-0}" != "1" ]; then
  bash "$GRAFT_REPO_ROOT/tools/pmc_passes.sh" "$TAG" || exit 1
fi
