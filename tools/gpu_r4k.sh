#!/bin/bash
# Round-4 final check: the whole GPU suite, smoke(), the default bench line,
# and a two-rank rehearsal of the multi-GPU bench path (gloo, both ranks on
# the one GPU).  Every step has its own limit; a failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_final.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_final.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $OUT/smoke_final.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py > $OUT/bench_final.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $OUT/bench_final.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --dist-backend gloo --steps 5 --warmup 2 --cpu-rays 0 --ref-gpu-rays 0 --no-alt > $OUT/bench_2rank.log 2>&1; rc=$?
echo "2-rank rc=$rc"; tail -1 $OUT/bench_2rank.log | cut -c1-300
