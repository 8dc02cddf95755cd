"""Print a rocprofv3 kernel_stats.csv as short name / calls / average us."""
import csv
import sys

for r in list(csv.DictReader(open(sys.argv[1])))[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    n = r["Name"]
    n = n[5:] if n.startswith("void ") else n
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{n[:60]:60s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:10.1f} us")
