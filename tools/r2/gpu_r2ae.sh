#!/bin/bash
# perturbed sampling on the fused path: new tests, render regressions, bench stage times
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_perturb.py tests/test_gpu_render.py tests/test_gpu_fullview.py > gpurun_out/r2ae_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|^E |passed|failed|perturbed|staged|whole" gpurun_out/r2ae_tests.log | cut -c1-250 | tail -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --no-alt --cpu-rays 0 --ref-gpu-rays 0 > gpurun_out/r2ae_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/r2ae_bench.log
