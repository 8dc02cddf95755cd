#!/bin/bash
# RGB training kernels: tests (gradient errors printed), step timing fused vs torch path, kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rgb_train.py > gpurun_out/r2s3h_tests.log 2>&1 || { tail -30 gpurun_out/r2s3h_tests.log; exit 1; }
grep -E "PASS|FAIL|relative" gpurun_out/r2s3h_tests.log | cut -c1-600
timeout -k 10 300 python -u tools/diag/rgb_train_time.py 4096 8192 > gpurun_out/r2s3h_time.log 2>&1 || { tail -20 gpurun_out/r2s3h_time.log; exit 1; }
cat gpurun_out/r2s3h_time.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2s3h" -o trace -- python3 "$GRAFT_REPO_ROOT/tools/diag/rgb_train_time.py" 8192 > "$GRAFT_REPO_ROOT/gpurun_out/r2s3h_trace.log" 2>&1 || { echo trace failed; exit 1; }
head -30 "$GRAFT_REPO_ROOT/gpurun_out/prof_r2s3h/trace_kernel_stats.csv" | cut -c1-400 | sed "s/(.*)//"
