set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/box_tests.log 2>&1; rc=$?; tail -1 $OUT/box_tests.log; [ $rc -ne 0 ] && tail -30 $OUT/box_tests.log && exit $rc
CASES='default X=0
direct SAMNERF_LOOKUP=packed' RS='8 4 16' bash tools/gpu_share_ab.sh
