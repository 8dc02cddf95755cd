#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
for cfg in "PF=1 REPS=6" "PF=1 SEG=2 REPS=6"; do
  env $cfg timeout -k 10 120 python -u tools/pf_diag.py > $OUT/pfd.txt 2>&1; rc=$?
  echo "== $cfg rc=$rc"; grep -v amdgpu.ids $OUT/pfd.txt | grep -v "^  \(w2\|samvit\|rows\|weights_sum\)" | cut -c1-160 | head -30; [ $rc -ne 0 ] && exit $rc
done
exit 0
