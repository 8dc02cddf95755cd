#!/bin/bash
# SAM head: LDS-DMA stream (product) vs VGPR-staged (diag build), alternating; and golden tests on the variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V="$GRAFT_REPO_ROOT/tools/diag/lib/head_stage.so"
SAMNERF_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_render.py -k "golden or bf16x3" > gpurun_out/r2ab_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r2ab_tests.log; [ $rc -ne 0 ] && exit $rc
for L in "" $V "" $V; do
SAMNERF_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-rays 0 --ref-gpu-rays 0 --no-alt > gpurun_out/r2ab.log 2>&1 || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/r2ab.log').read().splitlines()[-1])
print('${L:+staged}', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})
"
done
