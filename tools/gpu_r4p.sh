#!/bin/bash
# Round-4 batch p: attribution of the mask-training step -- the backward
# without its m_grid scatter (timing only) against the pipelined-dW build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/ab_train.sh 2 tools/bin/lib_dw.so tools/bin/lib_nosc.so || exit $?
