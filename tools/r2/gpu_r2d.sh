#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread tests/test_gpu_train.py > gpurun_out/r2d_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r2d_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r2d_tests.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --no-alt --cpu-rays 0 --ref-gpu-rays 0 --steps 20 > gpurun_out/r2d_bench.log 2>&1; rc=$?
python -c "import json;d=json.loads(open('gpurun_out/r2d_bench.log').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['stage_ms'])"
[ $rc -ne 0 ] && exit $rc
for a in "" "--torch-adam"; do timeout -k 10 200 python bench.py --mode train --steps 20 --warmup 5 $a > gpurun_out/r2d_train$a.log 2>&1 || exit $?; tail -c 700 gpurun_out/r2d_train$a.log; done
for v in pfpairs_old pfpairs; do for n in 70000 40000; do SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/diag/lib/$v.so timeout -k 10 200 python tools/diag/final_determinism.py $n > gpurun_out/r2d_det_${v}_$n.log 2>&1 || exit $?; echo "$v n=$n"; grep -E "repeat|image|rows" gpurun_out/r2d_det_${v}_$n.log; done; done
