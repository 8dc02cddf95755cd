#!/bin/bash
# fused proposal kernel: bit identity, then A/B timing (alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_render.py -k "proposal or golden or tiling or fullview" > gpurun_out/r2z_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/r2z_tests.log | head; [ $rc -ne 0 ] && exit $rc
for f in 1 0 1 0; do
SAMNERF_PROP_FUSED=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-rays 0 --ref-gpu-rays 0 --no-alt > gpurun_out/r2z.log 2>&1 || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/r2z.log').read().splitlines()[-1])
print('fused=$f', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})
"
done
