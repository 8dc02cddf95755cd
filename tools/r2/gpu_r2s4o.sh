#!/bin/bash
# k_rt_final_bwd: g1 in scratch (default: 104 VGPRs, 4 waves, 272 B/lane
# scratch) vs fully unrolled in registers (g1u.so: 206 VGPRs, 2 waves) vs
# unrolled at 3 waves (g1u3.so: 168 VGPRs, 56 spilled)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r2s4o; mkdir -p $R
for v in base g1u g1u3; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t_$v" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 20 --warmup 5 > "$R/t_$v.log" 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$R/t_$v/t_kernel_stats.csv')):
    if 'k_rt_final_bwd(' in r['Name'] or 'k_rt_final_bwdEN' in r['Name'] or r['Name'].startswith('(anonymous namespace)::k_rt_final_bwd('): print('$v', r['Name'][:40], float(r['AverageNs'])/1e3, 'us')"
done
echo ok
