#!/bin/bash
# Round-4 batch c: where the k_final prefetch form's renders differ
# (tools/pf_diag.py), the product build (mask head 5-deep DMA weight ring,
# s_grid per-level staging restored) through the mask / full-view / mask
# training GPU tests, then the headline and mask views timed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 200 python -u tools/pf_diag.py > $OUT/pf_diag.txt 2>&1; rc=$?
echo "pf_diag rc=$rc"; tail -30 $OUT/pf_diag.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_fullview.py tests/test_gpu_mask_train.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_c.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python bench.py --steps 30 --no-alt --cpu-rays 0 --ref-gpu-rays 0 > $OUT/bench_c.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $OUT/bench_c.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['stage_ms'])"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python tools/mask_view_time.py > $OUT/mask_c.log 2>&1; rc=$?; echo "mask rc=$rc"; tail -1 $OUT/mask_c.log
