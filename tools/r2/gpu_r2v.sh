#!/bin/bash
# A/B: ray tiles on/off, default-init and opaque-sphere scenes, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for sc in default surface; do
for a in "" "--no-tiles" "" "--no-tiles"; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-rays 0 --ref-gpu-rays 0 --no-alt --scene $sc $a > gpurun_out/r2v.log 2>&1 || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/r2v.log').read().splitlines()[-1])
print('$sc', '${a:-tiles}', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})
"
done; done
