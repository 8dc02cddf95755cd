#!/bin/bash
# Round-4 batch: parity of the candidate builds (s_grid DMA staging, replicated
# weight streams) through the GPU tests, then interleaved A/B timing.  Every
# GPU step has its own limit; a failure or timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
for L in lib_copies; do
  SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/bin/$L.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullview.py tests/test_gpu_render.py tests/test_gpu_mask.py tests/test_gpu_train.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$L.log 2>&1
  rc=$?; echo "pytest $L rc=$rc"; tail -2 $OUT/pytest_$L.log
  [ $rc -ne 0 ] && exit $rc
done
bash tools/ab_libs.sh 2 product tools/bin/lib_sgdma.so tools/bin/lib_copies.so || exit $?
bash tools/ab_mask.sh 2 tools/bin/lib_sgdma.so tools/bin/lib_copies.so tools/bin/lib_mnog.so tools/bin/lib_mnow.so tools/bin/lib_mnos.so || exit $?
