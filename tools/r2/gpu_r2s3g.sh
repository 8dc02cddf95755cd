#!/bin/bash
# drop-in grid backward on the torch RGB step's data: recorded vs permuted point order
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag/scatter_probe.py 8192 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r2s3g_probe.log
