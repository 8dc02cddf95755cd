#!/bin/bash
# A/B of the replicated coarse-level cap (SAMNERF_RT_REP_ROWS): step time and
# the scatter kernels' times per cap.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r2s4d; mkdir -p $R
for cap in 0 32768 60000 200000 600000; do
  SAMNERF_RT_REP_ROWS=$cap timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t_$cap" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 20 --warmup 5 > "$R/t_$cap.log" 2>&1 || { echo "trace $cap failed"; tail -5 "$R/t_$cap.log"; exit 1; }
  echo "== $cap"
done
for cap in 32768 600000; do
  SAMNERF_RT_REP_ROWS=$cap timeout -k 10 120 python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 30 --warmup 5 > "$R/b_$cap.log" 2>&1 || exit 1
  echo "bench $cap $(tail -1 $R/b_$cap.log | cut -c1-200)"
done
echo ok
