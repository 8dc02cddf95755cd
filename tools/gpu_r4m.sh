#!/bin/bash
# Round-4 batch m: attribution of the mask head's remaining time (timing-only
# builds: layer boundaries without leaky_relu / max / split; no m_grid gathers).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/ab_mask.sh 2 product tools/bin/lib_mnoepi.so tools/bin/lib_mnogat.so || exit $?
