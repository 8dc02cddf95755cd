#!/bin/bash
# Round-4 batch n: the mask GPU tests (incl. the ragged-launch case) on the
# rebuilt product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_mask_train.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_n.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|ragged|unfused_path" $OUT/pytest_n.log | tail -5; exit $rc
