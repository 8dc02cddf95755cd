#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rgb_train.py > gpurun_out/r2s3p_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r2s3p_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r2s3p_tests.log | head; exit $rc; }
timeout -k 10 300 python bench.py --mode rgbtrain --steps 20 --warmup 5 > gpurun_out/r2s3p_rgbtrain.log 2>&1 || { tail -20 gpurun_out/r2s3p_rgbtrain.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r2s3p_rgbtrain.log').read().splitlines()[-1]); print(d['ms_per_step'], d['torch_path_ms_per_step'], d['speedup_vs_torch_path'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2s3p" -o trace -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/r2s3p_trace.log" 2>&1 || { echo trace failed; exit 1; }
python3 "$GRAFT_REPO_ROOT/tools/summarize_trace.py" "$GRAFT_REPO_ROOT/gpurun_out/prof_r2s3p/trace_kernel_stats.csv" 16
