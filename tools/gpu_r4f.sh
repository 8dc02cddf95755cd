#!/bin/bash
# Round-4 batch f: the whole GPU suite on the product build (mask head: DMA
# weight ring + batched gathers; k_final without the prefetch form), then the
# mask view and the headline timed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_f.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_f.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python tools/mask_view_time.py > $OUT/mask_f.log 2>&1; rc=$?; echo "mask rc=$rc"; tail -1 $OUT/mask_f.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python bench.py --steps 30 --no-alt --cpu-rays 0 --ref-gpu-rays 0 > $OUT/bench_f.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $OUT/bench_f.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['stage_ms'])"
