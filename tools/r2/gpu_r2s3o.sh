#!/bin/bash
# RGB training bench on random-pixel rays (the reference's training batches) + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode rgbtrain --steps 20 --warmup 5 > gpurun_out/r2s3o_rgbtrain.log 2>&1 || { tail -20 gpurun_out/r2s3o_rgbtrain.log; exit 1; }
tail -1 gpurun_out/r2s3o_rgbtrain.log | cut -c1-420
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2s3o" -o trace -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/r2s3o_trace.log" 2>&1 || { echo trace failed; exit 1; }
python3 "$GRAFT_REPO_ROOT/tools/summarize_trace.py" "$GRAFT_REPO_ROOT/gpurun_out/prof_r2s3o/trace_kernel_stats.csv" 16
