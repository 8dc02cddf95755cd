#!/bin/bash
# Round-4 batch w: the mask head's first fragment pair of each weight step read
# before the previous step's barrier (finish() waits one step further ahead) --
# interleaved A/B of the mask view (ms, logits fingerprint) against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/lib_mpre.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_mpre.log 2>&1
rc=$?; echo "pytest mpre rc=$rc"; tail -1 $OUT/pytest_mpre.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_mask.sh 3 product tools/bin/lib_mpre.so || exit $?
