#!/bin/bash
# Round-4 batch t: the full GPU suite on the committed product, the mask
# training step's kernel trace (after the per-XCD coarse-level copies), and a
# default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/r4t_tests_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/r4t_tests_gpu.log; [ $rc -ne 0 ] && exit $rc
STEPS=20 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/r4t_mt -o mt -- python3 tools/mask_train_prof.py > $OUT/r4t_mt.log 2>&1
rc=$?; echo "mt prof rc=$rc"; tail -1 $OUT/r4t_mt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $OUT/r4t_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/r4t_bench.log; exit $rc; }
tail -1 $OUT/r4t_bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r.get('stage_ms'))"
