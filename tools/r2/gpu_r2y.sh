#!/bin/bash
# k_mask_head: product vs diagnostic variants (no gathers / no MFMAs / neither)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-product mask_nogather mask_nomfma mask_neither}; do
  if [ $v = product ]; then L=""; else L="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"; fi
  SAMNERF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2y_$v" -o m -- python3 -c "
import sys, torch
sys.path.insert(0, '$GRAFT_REPO_ROOT'); sys.path.insert(0, '$GRAFT_REPO_ROOT/segment-anything-nerf_amd')
import bench
bench.mask_view(torch.device('cuda', 0), 4, 1, 0, ref_rays=16384)
" > "$GRAFT_REPO_ROOT/gpurun_out/r2y_$v.log" 2>&1 || { echo "$v failed"; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/r2y_$v.log"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/prof_r2y_$v/m_kernel_stats.csv')):
    if 'k_mask_head' in r['Name'] or 'k_final' in r['Name']: print('$v', round(float(r['AverageNs'])/1e3,1), r['Name'][:60])
"
done
