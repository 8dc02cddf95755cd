#!/bin/bash
# full GPU suite, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -c "import __graft_entry__ as g; g.smoke()" && timeout -k 10 900 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r2t_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/r2t_tests.log | cut -c1-300 | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r2t_bench.log 2>&1 || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/r2t_bench.log').read().splitlines()[-1])
print('headline', round(d['value']/1e6,2), 'M rays/s', round(d['ms_per_step'],3), 'ms', {k:round(v,3) for k,v in d['stage_ms'].items()})
for k in ('n1_early_exit','precision_exact_fp32','cfg5_train','mask_default_head'):
    v=d.get(k) or {}; print(k, {a:(round(b,4) if isinstance(b,float) else b) for a,b in v.items() if a not in ('what','dtype','config','optimizer','data')})
"
