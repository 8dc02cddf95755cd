set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6g; mkdir -p $OUT
TAG=r6g STEPS="tests" PYTEST_ARGS="-s" PYTEST_FILES="tests/test_gpu_pdf_split.py" bash tools/gpu_run.sh || exit $?
grep -h "rays on the split path" $OUT/tests.log || true
AB_DIR=$OUT/ab bash tools/ab_libs.sh 3 product tools/bin/lib_pdfseq.so > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; [ $rc -ne 0 ] && exit $rc
AB_ARGS="--scene surface" AB_DIR=$OUT/ab_surface bash tools/ab_libs.sh 2 product tools/bin/lib_pdfseq.so > $OUT/ab_surface.log 2>&1; rc=$?; cat $OUT/ab_surface.log; [ $rc -ne 0 ] && exit $rc
AB_ARGS="--rank-share 8 --streams 3 --steps 60" AB_DIR=$OUT/ab_share bash tools/ab_libs.sh 2 product tools/bin/lib_pdfseq.so > $OUT/ab_share.log 2>&1; rc=$?; cat $OUT/ab_share.log; exit $rc
