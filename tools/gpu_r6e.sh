set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6e; mkdir -p $OUT
TAG=r6e STEPS="tests" bash tools/gpu_run.sh || exit $?
AB_DIR=$OUT/ab bash tools/ab_libs.sh 3 product tools/bin/lib_h16q.so > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/burst_clock.py > $OUT/burst.log 2>&1; rc=$?; cat $OUT/burst.log | tail -40; exit $rc
