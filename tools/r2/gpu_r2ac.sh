#!/bin/bash
# k_final segment form on both scenes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for sc in surface default; do for S in 1 2 4; do
SAMNERF_FINAL_S=$S timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-rays 0 --ref-gpu-rays 0 --no-alt --scene $sc > gpurun_out/r2ac.log 2>&1 || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/r2ac.log').read().splitlines()[-1])
print('$sc S=$S', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})
"
done; done
