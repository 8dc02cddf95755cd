#!/bin/bash
# cfg-5 distillation step: kernel trace and atomic requests
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_r2s3w" -o trace -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 20 --warmup 5 > "$OUT/r2s3w_trace.log" 2>&1 || { echo trace failed; tail -5 "$OUT/r2s3w_trace.log"; exit 1; }
python3 "$GRAFT_REPO_ROOT/tools/summarize_trace.py" "$OUT/prof_r2s3w/trace_kernel_stats.csv" 14
mkdir -p "$OUT/pmc_r2s3w"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_r2s3w/p0" -o p0 -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode train --steps 3 --warmup 1 > "$OUT/pmc_r2s3w/p0.log" 2>&1 || { echo pmc failed; exit 1; }
python3 - "$OUT/pmc_r2s3w" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/p0/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "GRBM_GUI_ACTIVE": n[k] += 1
for k in sorted(acc, key=lambda k: -acc[k]["TCC_EA0_ATOMIC_sum"])[:4]:
    c = n[k] or 1
    print(f"{k[:40]:40s} calls {c:3d}  atomic req/launch {acc[k]['TCC_EA0_ATOMIC_sum']/c:.3e}  us {acc[k]['GRBM_GUI_ACTIVE']/c/8/2.4e3:.1f}")
PY
