#!/bin/bash
# Round-2 evidence: default bench line, its kernel-trace stats, the PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r2final_bench.log 2>&1 || { tail -20 gpurun_out/r2final_bench.log; exit 1; }
tail -1 gpurun_out/r2final_bench.log > gpurun_out/r2final_bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_trace" -o trace -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 --no-alt --streams 1 > "$GRAFT_REPO_ROOT/gpurun_out/r2final_trace.log" 2>&1 || { echo trace failed; exit 1; }
cd "$GRAFT_REPO_ROOT"
bash tools/pmc_r2.sh r2final > gpurun_out/r2final_pmc.log 2>&1 || { tail -20 gpurun_out/r2final_pmc.log; exit 1; }
echo ok
