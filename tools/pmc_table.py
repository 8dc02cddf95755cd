#!/usr/bin/env python3
"""Per-kernel averages of every counter found under a pmc_probe.sh output dir."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    m = re.search(r"(k_\w+(<[^>]*>)?)", k)
    short = m.group(1) if m else k[:40]
    print(short, " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(vals[k].items())))
