#!/bin/bash
# Round-4 batch l: s_grid boxes staged by LDS DMA with a one-pass path for
# samples whose 4 boxes fit 64 slots each (SAMNERF_SGRID_SMALLBOX=1): parity
# (full-view corner rows and s_grid features) on that build, then interleaved
# A/B on the default and the sphere scene.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/lib_sbox.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fullview.py tests/test_gpu_render.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sbox.log 2>&1
rc=$?; echo "pytest sbox rc=$rc"; tail -2 $OUT/pytest_sbox.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh 2 product tools/bin/lib_sbox.so || exit $?
AB_ARGS="--scene surface" bash tools/ab_libs.sh 2 product tools/bin/lib_sbox.so || exit $?
