set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6i; mkdir -p $OUT
TAG=r6i STEPS="tests" PYTEST_ARGS="-s" PYTEST_FILES="tests/test_gpu_render.py tests/test_gpu_fullview.py tests/test_gpu_pdf_split.py" bash tools/gpu_run.sh || exit $?
AB_DIR=$OUT/ab bash tools/ab_libs.sh 3 product tools/bin/lib_rcpdiv.so > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
