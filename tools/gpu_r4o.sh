#!/bin/bash
# Round-4 batch o: the mask-training dW kernel with pipelined row loads (and
# 4,096-row chunks): its GPU tests, then interleaved A/B of the training step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
for L in lib_dw lib_dw4k; do
  SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mask_train.py tests/test_gpu_mask.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$L.log 2>&1
  rc=$?; echo "pytest $L rc=$rc"; tail -1 $OUT/pytest_$L.log; [ $rc -ne 0 ] && exit $rc
done
bash tools/ab_train.sh 2 product tools/bin/lib_dw.so tools/bin/lib_dw4k.so || exit $?
# attribution: the backward without its m_grid scatter (timing only)
bash tools/ab_train.sh 1 tools/bin/lib_dw.so tools/bin/lib_nosc.so || exit $?
