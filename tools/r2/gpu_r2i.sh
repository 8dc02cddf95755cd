#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread tests/test_gpu_train.py > gpurun_out/r2i_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|cfg5|Error" gpurun_out/r2i_tests.log | cut -c1-300; tail -2 gpurun_out/r2i_tests.log; [ $rc -ne 0 ] && { grep -B5 -A25 "def test_sgrid_backward_box" gpurun_out/r2i_tests.log | tail -40; exit $rc; }
for m in box corner; do SAMNERF_SGRID_BWD=$m timeout -k 10 200 python bench.py --mode train --steps 30 --warmup 5 > gpurun_out/r2i_train_$m.log 2>&1 || exit $?; python -c "import json;d=json.loads(open('gpurun_out/r2i_train_$m.log').read().splitlines()[-1]);print('$m', d['ms_per_step'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2i_train" -o train -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r2i_trainprof.log" 2>&1; echo "prof rc=$?"
