#!/bin/bash
# round 2: new parity tests + bench (headline, self-launched 2-rank rehearsal)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullview.py tests/test_gpu_dist.py > gpurun_out/r2a_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r2a_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r2a_bench.log 2>&1; rc=$?
tail -c 3000 gpurun_out/r2a_bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --dist-backend gloo --steps 4 --warmup 1 > gpurun_out/r2a_bench2.log 2>&1; rc=$?
tail -c 3000 gpurun_out/r2a_bench2.log
exit $rc
