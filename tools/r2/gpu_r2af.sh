#!/bin/bash
# box4 range reduction in lockstep + row broadcasts, 32-bit sample offsets: bit-identity tests, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_render.py tests/test_gpu_train.py tests/test_gpu_n1.py tests/test_gpu_fullview.py > gpurun_out/r2af_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/r2af_tests.log | cut -c1-250 | tail -20; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --no-alt --cpu-rays 0 --ref-gpu-rays 0 > gpurun_out/r2af_bench$i.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --steps 20 --no-alt --cpu-rays 0 --ref-gpu-rays 0 --scene surface > gpurun_out/r2af_bench_surf.log 2>&1 || exit $?
for f in gpurun_out/r2af_bench1.log gpurun_out/r2af_bench2.log gpurun_out/r2af_bench_surf.log; do python -c "
import json,sys;d=json.loads(open('$f').read().splitlines()[-1])
print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['stage_ms'].items()})"; done
