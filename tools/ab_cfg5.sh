#!/bin/bash
# Interleaved A/B of library builds on the config-5 distillation step
# (tools/cfg5_time.py).  usage (GPU box): bash tools/ab_cfg5.sh ROUNDS lib1 lib2 ...
set -o pipefail
ROUNDS=$1; shift
for r in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    tag=$(basename $L .so)
    if [ "$L" = product ]; then unset SAMNERF_LIB; else export SAMNERF_LIB="$GRAFT_REPO_ROOT/$L"; fi
    out=$(timeout -k 10 150 python tools/cfg5_time.py 2>/dev/null | tail -1); rc=$?
    if [ $rc -ne 0 ]; then echo "$tag round $r rc=$rc"; exit $rc; fi
    echo "cfg5 $tag $r $out"
  done
done
