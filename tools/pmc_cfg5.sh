#!/bin/bash
# the cfg-5 distillation step's s_grid scatter priced on
# the atomic path -- one rocprofv3 PMC pass (counters only) of bench.py
# --mode train: atomic wave-instructions (TD_ATOMIC_WAVEFRONT), memory-side
# atomic requests (TCC_EA0_ATOMIC) and their 32-B sectors (TCC_ATOMIC_SECTORS),
# per kernel; then tools/atomic_table.py.  usage (GPU box): bash tools/pmc_cfg5.sh TAG
set -o pipefail
TAG=${1:-cfg5}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TD_ATOMIC_WAVEFRONT_sum TCC_EA0_ATOMIC_sum TCC_ATOMIC_SECTORS_sum \
  GRBM_GUI_ACTIVE --output-format csv -d "$OUT/atom" -o atom -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 5 --warmup 2 > "$OUT/atom.log" 2>&1
rc=$?; echo "cfg5 atomic pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/atom.log"; exit $rc; }
python3 "$GRAFT_REPO_ROOT/tools/atomic_table.py" "$OUT/atom" | tee "$OUT/atomic_table.txt"
