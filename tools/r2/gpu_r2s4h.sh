#!/bin/bash
# Which s_grid levels the distillation step's scatter time comes from: builds
# whose k_sgrid_backward skips the levels below SG_DIAG_MINLEVEL (built with
# tools/diag/build_variant.sh sgK -DSG_DIAG_MINLEVEL=K), kernel times and
# atomic requests of bench --mode train per build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r2s4h; mkdir -p $R
for v in base sg1 sg3 sg6 sg16; do
  lib=""; [ $v != base ] && lib="$GRAFT_REPO_ROOT/tools/diag/lib/$v.so"
  SAMNERF_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/t_$v" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 20 --warmup 5 > "$R/t_$v.log" 2>&1 || { echo "trace $v failed"; tail -5 "$R/t_$v.log"; exit 1; }
  SAMNERF_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE --output-format csv -d "$R/p_$v" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 3 --warmup 1 > "$R/p_$v.log" 2>&1 || { echo "pmc $v failed"; tail -5 "$R/p_$v.log"; exit 1; }
  echo "== $v"
done
echo ok
