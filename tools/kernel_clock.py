#!/usr/bin/env python3
"""Shader clock per kernel from one rocprofv3 run holding both the
GRBM_GUI_ACTIVE counter and the kernel trace (tools/kernel_clock.sh): per
dispatch, GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / (End - Start),
averaged per kernel.  usage: python tools/kernel_clock.py <dir> [--json out.json]
(--json: the duration-weighted clock of each stage of the view, read by
bench.py's rooflines as profiles/kernel_clock.json)"""
import collections
import csv
import glob
import re
import sys


def main(root):
    dur = {}
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"])
    grbm = {}
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                grbm[r["Dispatch_Id"]] = float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for d, g in grbm.items():
        if d in dur and dur[d][0] > 0:
            m = re.search(r"(k_\w+(<[^>(]*>)?)", dur[d][1])
            per[m.group(1) if m else dur[d][1][:40]].append((g / 8.0 / dur[d][0], dur[d][0]))
    if "--json" in sys.argv:
        import json
        from pmc_rates import stage_of
        acc = collections.defaultdict(lambda: [0.0, 0.0])           # stage -> [sum clock*t, sum t]
        for d, g in grbm.items():
            if d in dur and dur[d][0] > 0:
                st = stage_of(dur[d][1])
                if st:
                    acc[st][0] += g / 8.0
                    acc[st][1] += dur[d][0]
        out = {"source": root, "what": "duration-weighted shader clock per stage: sum GRBM_GUI_ACTIVE / 8 / "
               "sum dispatch ns (tools/kernel_clock.py)",
               "stages": {st: a / t for st, (a, t) in acc.items() if t > 0}}
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    print(f"{'kernel':44s} {'dispatches':>10s} {'avg us':>8s} {'clock GHz':>9s}")
    for k, v in sorted(per.items(), key=lambda x: -sum(t for _, t in x[1])):
        print(f"{k[:44]:44s} {len(v):10d} {sum(t for _, t in v) / len(v) / 1e3:8.1f} "
              f"{sum(c for c, _ in v) / len(v):9.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
