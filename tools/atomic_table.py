#!/usr/bin/env python3
"""Per-kernel atomic counters of a rocprofv3 --pmc --kernel-trace run
(tools/pmc_cfg5.sh): dispatches, mean duration, atomic wave-instructions
(TD_ATOMIC_WAVEFRONT), memory-side atomic requests (TCC_EA0_ATOMIC), the
bytes they add (TCC_ATOMIC_SECTORS x 32 B) and that rate against the guide's
~1.3 TB/s of memory-side float-atomic adds (MI355X_MICROARCH.md "Global
float atomics").  usage: python tools/atomic_table.py <dir>"""
import collections
import csv
import glob
import re
import sys

ATOMIC_TBS = 1.3


def main(root):
    dur = {}
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+(<[^>(]*>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:40]
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            per[k]["_ns"].append(dur.get(r["Dispatch_Id"], 0))
    print(f"{'kernel':40s} {'us':>8s} {'atomic wave-inst':>17s} {'EA atomic req':>14s} {'bytes added':>12s} "
          f"{'TB/s':>6s} {'of 1.3':>7s}")
    for k, c in sorted(per.items(), key=lambda x: -sum(x[1].get("TD_ATOMIC_WAVEFRONT_sum", [0]))):
        td = c.get("TD_ATOMIC_WAVEFRONT_sum")
        if not td or max(td) == 0:
            continue
        n = len(td)
        ns = sum(c["_ns"]) / max(1, len(c["_ns"]))
        ea = sum(c.get("TCC_EA0_ATOMIC_sum", [0])) / n
        sec = sum(c.get("TCC_ATOMIC_SECTORS_sum", [0])) / n
        b = sec * 32.0
        tbs = b / (ns * 1e-9) / 1e12 if ns else 0.0
        print(f"{k[:40]:40s} {ns / 1e3:8.1f} {sum(td) / n:17.3e} {ea:14.3e} {b:12.3e} {tbs:6.2f} {tbs / ATOMIC_TBS:7.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
