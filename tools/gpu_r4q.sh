#!/bin/bash
# Round-4 batch q: mask-training scatter attribution by level range (timing
# only): levels 0-3 only, levels 4-15 only, none, all.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/ab_train.sh 2 product tools/bin/lib_sclo.so tools/bin/lib_schi.so tools/bin/lib_nosc.so || exit $?
