#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for a in "" "--no-tiles" "--streams 1"; do
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --cpu-rays 0 --ref-gpu-rays 0 $a > gpurun_out/r2u.log 2>&1 || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/r2u.log').read().splitlines()[-1])
p=d['precision_exact_fp32']; print('$a', p['max_abs_samvit_vs_headline'], p['max_abs_image_vs_headline'], round(d['ms_per_step'],3))
"
done
