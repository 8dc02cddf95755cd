#!/bin/bash
# kernel-trace stats of bench.py at a reduced view height (one rank's share)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
H=${1:-64}
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_h$H" -o t -- python "$GRAFT_REPO_ROOT/bench.py" --H $H --steps 20 --warmup 3 --cpu-rays 0 > "$OUT/prof_h$H.log" 2>&1 || exit $?
python - "$OUT/prof_h$H/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
