set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6o; mkdir -p $OUT
TAG=r6o STEPS="tests" PYTEST_ARGS="-s" PYTEST_FILES="tests/test_gpu_mask.py" bash tools/gpu_run.sh || exit $?
bash tools/ab_mask.sh 3 product tools/bin/lib_nopipe.so tools/bin/lib_mask32.so > $OUT/ab_mask.log 2>&1; rc=$?; cat $OUT/ab_mask.log; exit $rc
