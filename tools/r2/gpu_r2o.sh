#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread tests/test_gpu_train.py -k "head_train or cpu_twin or reduce_loss" > gpurun_out/r2o_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|head train|cfg5|^E " gpurun_out/r2o_tests.log | cut -c1-400 | head -40; tail -2 gpurun_out/r2o_tests.log; [ $rc -ne 0 ] && exit $rc
for hd in hip torch; do SAMNERF_TRAIN_HEAD=$hd timeout -k 10 200 python bench.py --mode train --steps 30 --warmup 5 > gpurun_out/r2o_train_$hd.log 2>&1 || exit $?; python -c "import json;d=json.loads(open('gpurun_out/r2o_train_$hd.log').read().splitlines()[-1]);print('$hd', round(d['ms_per_step'],3), d['final_loss'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2o_train" -o train -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r2o_trainprof.log" 2>&1; echo "prof rc=$?"
