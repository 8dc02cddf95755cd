#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2h_train" -o train -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r2h_train.log" 2>&1; rc=$?
echo "train prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2h_render" -o render -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 --no-alt --streams 1 > "$GRAFT_REPO_ROOT/gpurun_out/r2h_render.log" 2>&1; rc=$?
echo "render prof rc=$rc"; find "$GRAFT_REPO_ROOT/gpurun_out/prof_r2h_train" "$GRAFT_REPO_ROOT/gpurun_out/prof_r2h_render" -name "*stats*"
exit $rc
