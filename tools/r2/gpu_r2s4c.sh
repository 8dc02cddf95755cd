#!/bin/bash
# RGB training with the coarse levels' gradient in per-XCD copies: the RGB
# training tests, the step time, its kernel trace and atomic requests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-r2s4c}
timeout -k 10 600 python -u -m pytest -x -q -rA --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rgb_train.py > gpurun_out/${T}_tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/${T}_tests.log | cut -c1-300 | head -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode rgbtrain --steps 20 --warmup 5 > gpurun_out/${T}_rgbtrain.log 2>&1 || { tail -20 gpurun_out/${T}_rgbtrain.log; exit 1; }
tail -1 gpurun_out/${T}_rgbtrain.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/prof_${T}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 10 --warmup 3 > "$R.log" 2>&1 || { echo "trace failed"; tail -5 "$R.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE --output-format csv -d "${R}_pmc" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 3 --warmup 1 > "${R}_pmc.log" 2>&1 || { echo "pmc failed"; tail -5 "${R}_pmc.log"; exit 1; }
echo ok
