#!/bin/bash
# Round-4 batch u: what the s_grid scatter's levels cost in the config-5 step
# (timing-only builds that skip levels < 3 / all levels), interleaved A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/ab_cfg5.sh 3 product tools/bin/lib_sgmin3.so tools/bin/lib_sgmin16.so || exit $?
