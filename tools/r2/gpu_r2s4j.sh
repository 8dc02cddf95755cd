#!/bin/bash
# headline view rate vs the number of HIP streams views are issued on
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=gpurun_out/r2s4j; mkdir -p $R
for s in 1 2 3 4 2 3; do
  timeout -k 10 180 python bench.py --steps 40 --warmup 5 --cpu-rays 0 --ref-gpu-rays 0 --no-alt --streams $s > $R/s$s.log 2>&1 || { tail -5 $R/s$s.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$R/s$s.log').read().strip().splitlines()[-1]); print('streams', $s, round(d['value']/1e6,2), 'M rays/s', round(d['ms_per_step'],3), 'ms')"
done
echo ok
