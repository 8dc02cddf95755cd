#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2s" -o t -- python3 "$GRAFT_REPO_ROOT/tools/diag/tile_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/r2s.log" 2>&1; rc=$?
grep -v "rocprofv3\|^E20\|^W20" "$GRAFT_REPO_ROOT/gpurun_out/r2s.log" | tail -12; exit $rc
