set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6h; mkdir -p $OUT
TAG=r6h STEPS="tests" PYTEST_ARGS="-s" PYTEST_FILES="tests/test_gpu_pdf_split.py" bash tools/gpu_run.sh || exit $?
AB_DIR=$OUT/ab bash tools/ab_libs.sh 3 product tools/bin/lib_split64.so tools/bin/lib_pdfseq.so > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
