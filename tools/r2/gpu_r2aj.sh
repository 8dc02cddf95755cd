#!/bin/bash
# A/B on one box: previous commit (tools/diag/lib/prev.so) vs the tree (ReLU on float bits)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_render.py tests/test_gpu_fullview.py tests/test_gpu_train.py tests/test_gpu_mask.py tests/test_gpu_n1.py tests/test_perturb.py tests/test_gpu_encoders.py > gpurun_out/r2aj_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/r2aj_tests.log | cut -c1-250 | tail -20; [ $rc -ne 0 ] && exit $rc
for v in prev new prev new; do
  if [ $v = prev ]; then export SAMNERF_LIB=$PWD/tools/diag/lib/prev.so; else unset SAMNERF_LIB; fi
  timeout -k 10 300 python bench.py --steps 20 --no-alt --cpu-rays 0 --ref-gpu-rays 0 > gpurun_out/r2aj_bench_$v.log 2>&1 || exit $?
  python -c "
import json,sys;d=json.loads(open('gpurun_out/r2aj_bench_$v.log').read().splitlines()[-1])
print('$v', round(d['value']/1e6,2), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})"
done
