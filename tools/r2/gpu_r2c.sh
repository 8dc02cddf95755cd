#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_render.py > gpurun_out/r2c_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r2c_tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/r2c_tests.log; exit $rc; }
timeout -k 10 200 python bench.py --no-alt --cpu-rays 0 --ref-gpu-rays 0 --steps 20 > gpurun_out/r2c_bench.log 2>&1; rc=$?
python -c "import json;d=json.loads(open('gpurun_out/r2c_bench.log').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['stage_ms'])"
[ $rc -ne 0 ] && exit $rc
for n in 70000 40000; do SAMNERF_LIB=$GRAFT_REPO_ROOT/tools/diag/lib/pfpairs.so timeout -k 10 200 python tools/diag/final_determinism.py $n > gpurun_out/r2c_det_$n.log 2>&1 || exit $?; echo "pfpairs n=$n"; grep -E "repeat|image|rows" gpurun_out/r2c_det_$n.log; done
