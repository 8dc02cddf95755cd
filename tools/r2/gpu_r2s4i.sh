#!/bin/bash
# k_sgrid_backward with the levels interleaved in dispatch order vs the
# level-major launch (tools/diag/lib/sgmajor.so: -DSG_LEVEL_MAJOR=1): the
# distillation tests, then cfg-5 step time and the kernel's time per build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r2s4i
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py > gpurun_out/r2s4i/tests.log 2>&1; rc=$?
grep -E "FAILED|^E |passed|failed" gpurun_out/r2s4i/tests.log | cut -c1-300 | head; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r2s4i
for v in base sgmajor base sgmajor; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 40 --warmup 5 > "$R/b_$v.log" 2>&1 || exit 1
  echo "bench $v $(tail -1 $R/b_$v.log | cut -c1-170)"
done
for v in base sgmajor; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t_$v" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 20 --warmup 5 > "$R/t_$v.log" 2>&1 || exit 1
done
echo ok
