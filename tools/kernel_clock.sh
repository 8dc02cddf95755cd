#!/bin/bash
# Shader clock per kernel of the headline view: one rocprofv3 run with the
# GRBM_GUI_ACTIVE counter and the kernel trace (allowed together: no tracing
# domains), joined per dispatch by tools/kernel_clock.py
# (clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration).
# usage (GPU box): bash tools/kernel_clock.sh TAG [bench args]
set -o pipefail
TAG=${1:-clk}; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/clock_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d "$OUT" -o c -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --cpu-rays 0 --ref-gpu-rays 0 --no-alt --streams 1 "$@" > "$OUT/run.log" 2>&1
rc=$?; echo "clock run rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/run.log"; exit $rc; }
python3 "$GRAFT_REPO_ROOT/tools/kernel_clock.py" "$OUT"
