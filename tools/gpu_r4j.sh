#!/bin/bash
# Round-4 batch j: interleaved A/B of candidate builds -- s_grid at 5 waves per
# SIMD on the headline view, the mask weight ring 4 deep on the mask view.
# (Both variants also carry the hash-term-by-add change, measured separately:
# k_final 0.82 vs 0.81 ms, not kept; compare the s_grid / mask numbers.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/ab_libs.sh 2 product tools/bin/lib_sg5.so || exit $?
bash tools/ab_mask.sh 2 product tools/bin/lib_mr4.so || exit $?
