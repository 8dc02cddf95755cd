#!/bin/bash
# Round-4 batch x: k_final's exact zero-transmittance exit in the default mode
# (a wave stops once every ray's expf(-(float)cum) is 0): the render / N1 /
# full-view / training / dist tests on that build, then interleaved A/B of the
# headline view and of the opaque-sphere view against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/lib_zx.so timeout -k 10 500 python -u -m pytest tests/test_gpu_n1.py tests/test_gpu_render.py tests/test_gpu_fullview.py tests/test_gpu_train.py tests/test_gpu_dist.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_zx.log 2>&1
rc=$?; echo "pytest zx rc=$rc"; tail -1 $OUT/pytest_zx.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh 3 product tools/bin/lib_zx.so || exit $?
AB_ARGS="--scene surface" bash tools/ab_libs.sh 3 product tools/bin/lib_zx.so || exit $?
