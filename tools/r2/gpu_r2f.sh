#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in pfpairs_old_wz pfpairs_old; do n=70000; SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/diag/lib/$v.so timeout -k 10 200 python tools/diag/final_determinism.py $n > gpurun_out/r2f_det_${v}_$n.log 2>&1 || exit $?; echo "$v n=$n"; grep -E "repeat|image|rows" gpurun_out/r2f_det_${v}_$n.log; done
