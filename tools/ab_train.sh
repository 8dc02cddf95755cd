#!/bin/bash
# Interleaved A/B of library builds on the --with_mask training step
# (tools/mask_train_prof.py).  usage (GPU box): bash tools/ab_train.sh ROUNDS lib1 lib2 ...
set -o pipefail
ROUNDS=$1; shift
for r in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    tag=$(basename $L .so)
    if [ "$L" = product ]; then unset SAMNERF_LIB; else export SAMNERF_LIB="$GRAFT_REPO_ROOT/$L"; fi
    out=$(timeout -k 10 150 python tools/mask_train_prof.py 2>/dev/null | tail -1); rc=$?
    if [ $rc -ne 0 ]; then echo "$tag round $r rc=$rc"; exit $rc; fi
    echo "train $tag $r $out"
  done
done
