#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mask.py > gpurun_out/r2aa_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r2aa_tests.log; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/r2aa_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "
import sys, json, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'segment-anything-nerf_amd')
import bench
for hm in (0, 1):
    d = bench.mask_view(torch.device('cuda', 0), 6, 2, hm)
    d.pop('what'); d.pop('dtype'); print(hm, json.dumps(d))
" 2>&1 | grep -v amdgpu.ids
