#!/bin/bash
# fused mask head: timing and kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -c "
import sys, json, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'segment-anything-nerf_amd')
import bench
for hm in (0, 1):
    d = bench.mask_view(torch.device('cuda', 0), 6, 2, hm)
    d.pop('what'); d.pop('dtype'); print(hm, json.dumps(d))
" > gpurun_out/r2x.log 2>&1 || { tail -20 gpurun_out/r2x.log; exit 1; }
cat gpurun_out/r2x.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2x" -o m -- python3 -c "
import sys, torch
sys.path.insert(0, '$GRAFT_REPO_ROOT'); sys.path.insert(0, '$GRAFT_REPO_ROOT/segment-anything-nerf_amd')
import bench
bench.mask_view(torch.device('cuda', 0), 4, 1, 0, ref_rays=16384)
" > "$GRAFT_REPO_ROOT/gpurun_out/r2x_prof.log" 2>&1; echo "prof rc=$?"
