#!/bin/bash
# A/B of the number of gradient copies for the replicated levels (8 / 16 / 32)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r2s4e; mkdir -p $R
for v in base krep16 krep32 base; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 40 --warmup 5 > "$R/b_$v.log" 2>&1 || exit 1
  echo "bench $v $(tail -1 $R/b_$v.log | cut -c1-160)"
done
SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/diag/lib/krep16.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t16" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 20 --warmup 5 > "$R/t16.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t8" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 20 --warmup 5 > "$R/t8.log" 2>&1 || exit 1
echo ok
