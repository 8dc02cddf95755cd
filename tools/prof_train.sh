#!/bin/bash
# cfg-5 training step: bench line + kernel-trace stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 > "$OUT/bench_train.log" 2>&1 || { tail -20 "$OUT/bench_train.log"; exit 1; }
tail -1 "$OUT/bench_train.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_train" -o t -- python "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 10 --warmup 2 > "$OUT/prof_train.log" 2>&1 || exit $?
python - "$OUT/prof_train/t_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:18]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Percentage"])
PY
