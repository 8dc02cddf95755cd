#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rgb_train.py > gpurun_out/r2s3k_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|^E " gpurun_out/r2s3k_tests.log | cut -c1-300 | head -30; exit $rc
