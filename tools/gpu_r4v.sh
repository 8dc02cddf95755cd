#!/bin/bash
# Round-4 batch v: the s_grid scatter with a sample's surviving lanes packed
# into fewer atomic instructions (thresholds 256 / 384 / 512 of 512 lanes):
# the training tests on the always-packing build, then interleaved A/B of the
# config-5 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/lib_cmp512.so timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_cmp.log 2>&1
rc=$?; echo "pytest cmp512 rc=$rc"; tail -1 $OUT/pytest_cmp.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_cfg5.sh 3 product tools/bin/lib_cmp256.so tools/bin/lib_cmp384.so tools/bin/lib_cmp512.so || exit $?
