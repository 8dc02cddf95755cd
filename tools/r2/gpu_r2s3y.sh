#!/bin/bash
# atomic requests of the RGB training kernels (one PMC pass, counters only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_r2s3y"; mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p0" -o p0 -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode rgbtrain --steps 3 --warmup 1 > "$OUT/p0.log" 2>&1; rc=$?
echo "rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p0.log"; exit $rc; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/p0/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "GRBM_GUI_ACTIVE": n[k] += 1
for k in sorted(acc, key=lambda k: -acc[k]["TCC_EA0_ATOMIC_sum"])[:8]:
    c = n[k] or 1
    print(f"{k[:40]:40s} calls {c:3d}  atomic req/launch {acc[k]['TCC_EA0_ATOMIC_sum']/c:.3e}  GRBM/launch {acc[k]['GRBM_GUI_ACTIVE']/c:.3e}")
PY
