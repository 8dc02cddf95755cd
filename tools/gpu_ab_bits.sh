#!/bin/bash
# Bit identity + interleaved timing of the product against one A/B build:
#   TAG=... LIB=tools/bin/lib_X.so [AB_ROUNDS=3] [MASK=1] bash tools/gpu_ab_bits.sh   (GPU box)
# tools/lib_bits.py fingerprints for both (they must match), then
# tools/ab_scenes.sh (default + sphere scene) and, with MASK=1, tools/ab_mask.sh.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 240 python tools/lib_bits.py > $OUT/bits_product.json 2> $OUT/bits_product.err &&
SAMNERF_LIB=$GRAFT_REPO_ROOT/$LIB timeout -k 10 240 python tools/lib_bits.py > $OUT/bits_ab.json 2> $OUT/bits_ab.err &&
cat $OUT/bits_product.json $OUT/bits_ab.json &&
(cmp -s $OUT/bits_product.json $OUT/bits_ab.json && echo BITS IDENTICAL || echo BITS DIFFER) &&
AB_ROUNDS=${AB_ROUNDS:-3} bash tools/ab_scenes.sh product $LIB > $OUT/ab_scenes.txt 2>&1 &&
if [ "${MASK:-0}" = 1 ]; then bash tools/ab_mask.sh 2 product $LIB > $OUT/ab_mask.txt 2>&1; fi
