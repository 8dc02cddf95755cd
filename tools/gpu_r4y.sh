#!/bin/bash
# Round-4 batch y (final): smoke, the full GPU suite and a default bench line on
# the committed tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r4y_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/r4y_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r4y_tests_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/r4y_tests_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $OUT/r4y_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/r4y_bench.log; exit $rc; }
tail -1 $OUT/r4y_bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r.get('stage_ms'))"
