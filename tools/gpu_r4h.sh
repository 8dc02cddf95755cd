#!/bin/bash
# Round-4 batch h: kernel trace of the --with_mask training step and of the
# mask view (where the 3.2 ms and the 6.5 ms go).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_mtrain" -o mt -- \
  python3 "$GRAFT_REPO_ROOT/tools/mask_train_prof.py" > "$OUT/prof_mtrain.log" 2>&1; rc=$?
echo "mtrain rc=$rc"; tail -1 "$OUT/prof_mtrain.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_mview" -o mv -- \
  python3 "$GRAFT_REPO_ROOT/tools/mask_view_time.py" > "$OUT/prof_mview.log" 2>&1; rc=$?
echo "mview rc=$rc"; tail -1 "$OUT/prof_mview.log"
