#!/bin/bash
# tools/ab_libs.sh on the default and the opaque-sphere scene.  usage (GPU box):
#   AB_ROUNDS=2 bash tools/ab_scenes.sh lib1 lib2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
AB_DIR="$GRAFT_REPO_ROOT/gpurun_out/abs_default" bash tools/ab_libs.sh ${AB_ROUNDS:-2} "$@" || exit $?
AB_ARGS="--scene surface" AB_DIR="$GRAFT_REPO_ROOT/gpurun_out/abs_surface" bash tools/ab_libs.sh ${AB_ROUNDS:-2} "$@" | sed 's/^/surface /'
