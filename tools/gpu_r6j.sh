set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6j; mkdir -p $OUT
AB_DIR=$OUT/ab bash tools/ab_libs.sh 3 product tools/bin/lib_prop6.so tools/bin/lib_sg5.so > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
