#!/bin/bash
# Interleaved A/B of library builds on the --with_mask 512x512 view
# (tools/mask_view_time.py).  usage (GPU box): bash tools/ab_mask.sh ROUNDS lib1 lib2 ...
set -o pipefail
ROUNDS=$1; shift
for r in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    tag=$(basename $L .so)
    if [ "$L" = product ]; then unset SAMNERF_LIB; else export SAMNERF_LIB="$GRAFT_REPO_ROOT/$L"; fi
    out=$(timeout -k 10 120 python tools/mask_view_time.py 2>/dev/null | tail -1); rc=$?
    if [ $rc -ne 0 ]; then echo "$tag round $r rc=$rc"; exit $rc; fi
    echo "mask $tag $r $out"
  done
done
