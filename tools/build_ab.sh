#!/bin/bash
# Build a timing variant of the whole library into tools/bin/lib_<tag>.so
# (A/B of two builds in one GPU session via SAMNERF_LIB): usage
#   bash tools/build_ab.sh TAG [-DMACRO ...]     (run from the repo root)
set -e
TAG=$1; shift
OUT=tools/bin/obj_$TAG
mkdir -p $OUT
SRC=segment-anything-nerf_amd/csrc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -I include $*"
pids=()
for f in common.cpp grid_encoder.hip sh_freq_encoder.hip raymarch.hip sam_head.hip tile_codec.hip train_optim.hip sam_head_train.hip mask_head.hip rgb_train.hip mask_head_train.hip; do
  if [ "${f##*.}" = cpp ]; then X="-x hip"; else X=""; fi
  hipcc $X $FLAGS -c $SRC/$f -o $OUT/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
hipcc --offload-arch=gfx950 -shared -fPIC -o tools/bin/lib_$TAG.so $OUT/*.o
rm -rf $OUT
echo tools/bin/lib_$TAG.so
