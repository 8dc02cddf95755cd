#!/bin/bash
# Round-4 batch s: the mask head's layer-boundary max taken from the raw
# accumulators (leaky_relu moved to the splits) -- its GPU tests, then an
# interleaved A/B of the mask view (ms, logits fingerprint) against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/lib_mmax.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_mmax.log 2>&1
rc=$?; echo "pytest mmax rc=$rc"; tail -1 $OUT/pytest_mmax.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_mask.sh 3 product tools/bin/lib_mmax.so || exit $?
