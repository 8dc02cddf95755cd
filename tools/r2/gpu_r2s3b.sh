#!/bin/bash
# RGB training kernels: the new GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -rA --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rgb_train.py > gpurun_out/r2s3b_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert|^E " gpurun_out/r2s3b_tests.log | cut -c1-400 | head -40; exit $rc
