#!/bin/bash
# Round-4 batch i: mask head with the two-instruction leaky relu -- its GPU
# tests (inference, training, determinism) and the mask view timed twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_mask_train.py tests/test_gpu_render.py -k "mask or deterministic" -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_i.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_i.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 150 python tools/mask_view_time.py > $OUT/mask_i.log 2>&1; rc=$?; echo "mask rc=$rc"; tail -1 $OUT/mask_i.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
