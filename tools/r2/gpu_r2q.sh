#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2q" -o n1 -- python3 "$GRAFT_REPO_ROOT/tools/diag/n1_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/r2q.log" 2>&1; rc=$?
tail -3 "$GRAFT_REPO_ROOT/gpurun_out/r2q.log"; exit $rc
