#!/bin/bash
# Round-4 measurement set b (GPU box): headline-only kernel trace, the six PMC
# passes of the headline view, the cache passes of the opaque-sphere scene, and
# the default bench line.  Every step has its own limit; a failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
SKIP_PMC=1 bash tools/prof_r4.sh r4b || exit $?
bash tools/pmc_passes.sh r4b || exit $?
PASSES="4 5" bash tools/pmc_passes.sh r4bsurf --scene surface || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 420 python bench.py > $OUT/bench_r4b.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $OUT/bench_r4b.log | cut -c1-400
