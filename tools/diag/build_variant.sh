#!/bin/bash
# Build a diagnostic variant of libsamnerf_hip.so with extra -D flags into
# tools/diag/lib/<name>.so (load it with SAMNERF_LIB=...).
# usage: bash tools/diag/build_variant.sh NAME -DFOO=1 ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
SRC=$ROOT/segment-anything-nerf_amd/csrc
OUT=$ROOT/tools/diag/lib
OBJ=$(mktemp -d)
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -I $ROOT/include $*"
for f in common.cpp grid_encoder.hip sh_freq_encoder.hip raymarch.hip sam_head.hip tile_codec.hip train_optim.hip sam_head_train.hip mask_head.hip rgb_train.hip; do
  x=""; [[ $f == *.cpp ]] && x="-x hip"
  /opt/rocm/bin/hipcc $x $FLAGS -c $SRC/$f -o $OBJ/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/$NAME.so $OBJ/*.o
rm -rf $OBJ
echo "built $OUT/$NAME.so"
