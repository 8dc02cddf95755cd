#!/bin/bash
# Scatter lane order: atomic instruction q takes samples 16q .. 16q+15 (default:
# consecutive samples of a ray share 64-B segments at the dense levels) vs
# samples q, q+4, ... (tools/diag/lib/quadil.so: -DRT_QUAD_INTERLEAVED=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r2s4l
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rgb_train.py > gpurun_out/r2s4l/tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/r2s4l/tests.log | cut -c1-300 | head; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r2s4l
for v in base quadil base quadil; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 40 --warmup 5 > "$R/b_$v.log" 2>&1 || exit 1
  echo "bench $v $(tail -1 $R/b_$v.log | cut -c1-170)"
done
for v in base quadil; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t_$v" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 20 --warmup 5 > "$R/t_$v.log" 2>&1 || exit 1
  SAMNERF_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE --output-format csv -d "$R/p_$v" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 3 --warmup 1 > "$R/p_$v.log" 2>&1 || exit 1
done
echo ok
