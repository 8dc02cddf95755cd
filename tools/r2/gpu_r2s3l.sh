#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rgb_train.py tests/test_gpu_train.py tests/test_perturb.py tests/test_gpu_mask.py > gpurun_out/r2s3l_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|^E " gpurun_out/r2s3l_tests.log | cut -c1-300 | tail -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode rgbtrain --steps 20 --warmup 5 > gpurun_out/r2s3l_rgbtrain.log 2>&1 || { tail -20 gpurun_out/r2s3l_rgbtrain.log; exit 1; }
tail -1 gpurun_out/r2s3l_rgbtrain.log | cut -c1-400
