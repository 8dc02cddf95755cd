#!/bin/bash
# Which grid levels the RGB training scatters' atomic requests come from:
# builds that skip some levels' scatter (tools/diag/build_variant.sh with
# RT_DIAG_LMASK / RT_DIAG_PMASK, built first with e.g. `bash tools/diag/build_variant.sh
# lm0003 -DRT_DIAG_LMASK=0xFFFC`), per build the kernel times and the atomic
# request count of one bench --mode rgbtrain run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r2s4b
R=$GRAFT_REPO_ROOT/gpurun_out/r2s4b
cd /tmp && export TMPDIR=/tmp
for v in base lm0003 lm003f pm01 lmall; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t_$v" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 10 --warmup 3 > "$R/t_$v.log" 2>&1 || { echo "trace $v failed"; tail -5 "$R/t_$v.log"; exit 1; }
  SAMNERF_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE --output-format csv -d "$R/p_$v" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 3 --warmup 1 > "$R/p_$v.log" 2>&1 || { echo "pmc $v failed"; tail -5 "$R/p_$v.log"; exit 1; }
  echo "== $v"; tail -1 "$R/t_$v.log" | cut -c1-200
done
echo ok
