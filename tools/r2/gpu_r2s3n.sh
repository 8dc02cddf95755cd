#!/bin/bash
# s_grid scatter along-ray merge: tests, cfg-5 step A/B (corner vs run, and run on coarse levels only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_encoders.py > gpurun_out/r2s3n_tests.log 2>&1; rc=$?
grep -E "scatter|passed|failed|^E " gpurun_out/r2s3n_tests.log | head; [ $rc -ne 0 ] && exit $rc
for v in corner run64 run128 run; do
  case $v in corner) E="SAMNERF_SGRID_BWD=corner";; run64) E="SAMNERF_SGRID_RUN_RES=64";; run128) E="SAMNERF_SGRID_RUN_RES=128";; run) E="X=1";; esac
  env $E timeout -k 10 200 python bench.py --mode train --steps 30 --warmup 5 > gpurun_out/r2s3n_train_$v.log 2>&1 || { tail -5 gpurun_out/r2s3n_train_$v.log; exit 1; }
  echo $v $(tail -1 gpurun_out/r2s3n_train_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'ms', round(d['final_loss'],5))")
done
