#!/bin/bash
# SAM head lazy-epilogue variant (tools/diag/lib/head_lazy.so) vs the default: golden tests, alternating bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/tools/diag/lib/head_lazy.so
SAMNERF_LIB=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_render.py > gpurun_out/r2s3r_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r2s3r_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r2s3r_tests.log | head; exit $rc; }
for i in 1 2 3; do
  for v in base lazy; do
    if [ $v = lazy ]; then E="SAMNERF_LIB=$L"; else E="X=1"; fi
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-alt --cpu-rays 0 --ref-gpu-rays 0 > gpurun_out/r2s3r_$v$i.log 2>&1 || { tail -5 gpurun_out/r2s3r_$v$i.log; exit 1; }
    echo $v $i $(tail -1 gpurun_out/r2s3r_$v$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), {k:round(x,4) for k,x in d['stage_ms'].items()})")
  done
done
