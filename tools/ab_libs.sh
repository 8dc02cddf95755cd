#!/bin/bash
# Interleaved A/B of whole library builds on the headline view: for each round,
# for each library (a path, or "product" for the in-tree build), one
# `bench.py --no-alt` run with SAMNERF_LIB pointing at it; prints ms/view and
# stage ms.  usage (GPU box): bash tools/ab_libs.sh ROUNDS lib1 lib2 ...
set -o pipefail
ROUNDS=$1; shift
OUT="${AB_DIR:-$GRAFT_REPO_ROOT/gpurun_out/ab}"
mkdir -p "$OUT"
for r in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    tag=$(basename $L .so)
    if [ "$L" = product ]; then unset SAMNERF_LIB; else export SAMNERF_LIB="$GRAFT_REPO_ROOT/$L"; fi
    timeout -k 10 120 python bench.py --steps 30 --no-alt --cpu-rays 0 --ref-gpu-rays 0 ${AB_ARGS:-} > "$OUT/${tag}_$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag round $r rc=$rc"; tail -3 "$OUT/${tag}_$r.log"; exit $rc; fi
    tail -1 "$OUT/${tag}_$r.log" | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$tag', $r, round(r['ms_per_step'],4), {k: round(v,4) for k,v in r['stage_ms'].items()}, 'clock', r['config'].get('timed_clock_ghz'), 'views_in_flight', r['config'].get('views_in_flight'))"
  done
done
