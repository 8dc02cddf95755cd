set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_all.log 2>&1; rc=$?; tail -2 $OUT/pytest_all.log
[ $rc -ne 0 ] && grep -E "FAILED|Error" $OUT/pytest_all.log | head && exit $rc
timeout -k 10 200 python bench.py --mode gui --steps 30 > $OUT/bench_gui.log 2>&1; echo "gui rc=$?"; tail -1 $OUT/bench_gui.log
timeout -k 10 200 python bench.py --no-sam --cpu-rays 65536 > $OUT/bench_rgb.log 2>&1; echo "rgb rc=$?"; tail -1 $OUT/bench_rgb.log | cut -c1-700
