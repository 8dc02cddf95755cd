#!/bin/bash
# Round-4 batch r: mask training with the coarse m_grid levels scattered into
# per-XCD gradient copies -- its GPU tests, then interleaved A/B of the step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/lib_rep.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mask_train.py tests/test_gpu_mask.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_rep.log 2>&1
rc=$?; echo "pytest rep rc=$rc"; tail -1 $OUT/pytest_rep.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_train.sh 3 product tools/bin/lib_rep.so || exit $?
