#!/bin/bash
# fused mask head: tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread tests/test_gpu_mask.py tests/test_gpu_render.py > gpurun_out/r2w_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed|fused mask|adaptive|^[01] (image|weights|instance)" gpurun_out/r2w_tests.log | cut -c1-300 | head -30; exit $rc
