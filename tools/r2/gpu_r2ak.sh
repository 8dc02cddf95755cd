#!/bin/bash
# proposal gathers: direct (default) vs the box form (SAMNERF_LOOKUP=box) after the cheaper box lookups
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in direct box direct box; do
  if [ $v = box ]; then export SAMNERF_LOOKUP=box; else unset SAMNERF_LOOKUP; fi
  timeout -k 10 300 python bench.py --steps 20 --no-alt --cpu-rays 0 --ref-gpu-rays 0 > gpurun_out/r2ak_bench_$v.log 2>&1 || exit $?
  python -c "
import json,sys;d=json.loads(open('gpurun_out/r2ak_bench_$v.log').read().splitlines()[-1])
print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})"
done
