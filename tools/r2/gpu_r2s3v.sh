#!/bin/bash
# s_grid scatter with paired corner emission: tests, cfg-5 step, atomic requests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_train.py > gpurun_out/r2s3v_tests.log 2>&1; rc=$?
grep -E "scatter|passed|failed|^E " gpurun_out/r2s3v_tests.log | head; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --mode train --steps 30 --warmup 5 > gpurun_out/r2s3v_train$i.log 2>&1 || { tail -5 gpurun_out/r2s3v_train$i.log; exit 1; }
echo train $(tail -1 gpurun_out/r2s3v_train$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'ms', round(d['final_loss'],5))")
done
bash tools/r2/gpu_r2s3w.sh
