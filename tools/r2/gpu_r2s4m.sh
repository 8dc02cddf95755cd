#!/bin/bash
# k_rt_final_fwd at 3 waves per SIMD (now the default; fw3.so was built with -DRT_FWD_WAVES=3,
# 168 VGPRs, no spills) vs the compiler's 186 VGPRs (2 waves)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r2s4m; mkdir -p $R
for v in base fw3; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t_$v" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 20 --warmup 5 > "$R/t_$v.log" 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$R/t_$v/t_kernel_stats.csv')):
    if 'k_rt_final_fwd' in r['Name']: print('$v k_rt_final_fwd', float(r['AverageNs'])/1e3, 'us')"
done
echo ok
