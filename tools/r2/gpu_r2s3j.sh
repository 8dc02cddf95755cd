#!/bin/bash
# full GPU suite after the RGB training kernels, bench --mode rgbtrain, default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r2s3j_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/r2s3j_tests.log | cut -c1-300 | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode rgbtrain --steps 20 --warmup 5 > gpurun_out/r2s3j_rgbtrain.log 2>&1 || { tail -20 gpurun_out/r2s3j_rgbtrain.log; exit 1; }
tail -1 gpurun_out/r2s3j_rgbtrain.log
timeout -k 10 600 python bench.py > gpurun_out/r2s3j_bench.log 2>&1 || { tail -20 gpurun_out/r2s3j_bench.log; exit 1; }
tail -1 gpurun_out/r2s3j_bench.log > gpurun_out/r2s3j_bench.jsonl
python -c "
import json;d=json.loads(open('gpurun_out/r2s3j_bench.jsonl').read())
print('headline', round(d['value']/1e6,2), 'M rays/s', round(d['ms_per_step'],3), 'ms', {k:round(v,3) for k,v in d['stage_ms'].items()})
print('rgb_train', {a:(round(b,4) if isinstance(b,float) else b) for a,b in d['rgb_train'].items() if a not in ('dtype','data','config')})
"
