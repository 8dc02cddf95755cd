#!/bin/bash
# k_final S = 2 / 4 forms (one rank's share): packed corner weights in the scalar-FMA finish; A/B vs prev
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_render.py > gpurun_out/r2al_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/r2al_tests.log | cut -c1-250 | tail -20; [ $rc -ne 0 ] && exit $rc
for v in prev new prev new; do
  if [ $v = prev ]; then export SAMNERF_LIB=$PWD/tools/diag/lib/prev.so; else unset SAMNERF_LIB; fi
  for rs in 8 4; do
  timeout -k 10 300 python bench.py --steps 30 --no-alt --cpu-rays 0 --ref-gpu-rays 0 --rank-share $rs > gpurun_out/r2al_bench_${v}_$rs.log 2>&1 || exit $?
  python -c "
import json,sys;d=json.loads(open('gpurun_out/r2al_bench_${v}_$rs.log').read().splitlines()[-1])
print('$v share $rs', round(d['value']/1e6,2), round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['stage_ms'].items()})"
  done
done
