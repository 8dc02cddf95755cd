#!/bin/bash
# N1 early exit + checkpoint render + head-train tests, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread tests/test_gpu_n1.py tests/test_gpu_render.py  > gpurun_out/r2p_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|N1|surface|^E " gpurun_out/r2p_tests.log | cut -c1-400 | head -40; tail -2 gpurun_out/r2p_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r2p_bench.log 2>&1 || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/r2p_bench.log').read().splitlines()[-1])
print('headline', round(d['value']/1e6,2), 'M rays/s', round(d['ms_per_step'],3), 'ms', d['stage_ms'])
for k in ('n1_early_exit','precision_exact_fp32','cfg5_train'):
    v=d.get(k); print(k, {a:b for a,b in (v or {}).items() if a not in ('what',)})
"
