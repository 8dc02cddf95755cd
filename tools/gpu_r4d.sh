#!/bin/bash
# Round-4 batch d: tools/pf_diag.py over the k_final forms (which renders of
# a fresh process differ, and where), then the pipelined mask head's GPU
# tests and mask-view time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
for cfg in "PF=0" "PF=1 NEWFR=1" "PF=1 HEAD_MODE=1" "PF=0 SEG=2" "PF=1 SEG=2"; do
  env $cfg timeout -k 10 120 python -u tools/pf_diag.py > $OUT/pfd.txt 2>&1; rc=$?
  echo "== $cfg rc=$rc"; grep -v amdgpu.ids $OUT/pfd.txt | cut -c1-200 | head -12; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_mask.py tests/test_gpu_mask_train.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_d.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python tools/mask_view_time.py > $OUT/mask_d.log 2>&1; rc=$?; echo "mask rc=$rc"; tail -1 $OUT/mask_d.log
