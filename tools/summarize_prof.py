#!/usr/bin/env python3
"""Summarise rocprofv3 outputs (gpurun_out/prof_*) into profiles/.

  profiles/<tag>_kernel_stats.csv  -- rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.csv           -- per-kernel FETCH_SIZE / WRITE_SIZE averages
  profiles/pmc_traffic.json        -- {stage: HBM bytes per launch} read by bench.py

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC EA requests).  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE reads 1/2 of the bytes of a WIDE
(16 B/lane) coalesced stream and WRITE_SIZE is exact for 16-B stores; the
gathers here are 8-32 B per lane, a width the guide lists as uncalibrated.
`hbm_bytes` applies the guide's correction (2 * FETCH + WRITE); the raw fetch
is kept beside it.  Passes are separate runs (FETCH_SIZE needs 3 TCC slots,
WRITE_SIZE 2).
usage: python tools/summarize_prof.py --tag r1 [--pmc-dir pmc]
"""
import argparse
import collections
import csv
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")

STAGE_OF = {"k_snf": "prop0", "k_prop_sigma<128": "prop0", "k_prop_pdf<128": "prop0",
            "k_prop_sigma<64": "prop1", "k_prop_pdf<64": "prop1", "k_final": "final",
            "k_sgrid<": "s_grid", "k_sgrid_box4": "s_grid", "k_sam_head": "sam_head", "k_pack": "sam_head",
            "k_get_rays": "get_rays", "k_put_tables": "tables"}


def stage(name):
    for k, v in STAGE_OF.items():
        if k in name:
            return v
    return None


def pmc(root, counter):
    """Per-kernel average of `counter` over every counter_collection.csv
    under `root` (one rocprofv3 --pmc pass per directory)."""
    import glob
    d = collections.defaultdict(list)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter:
                d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r1")
    ap.add_argument("--pmc-dir", default="pmc", help="under gpurun_out/ (tools/gpu_ab.sh writes pmc/)")
    a = ap.parse_args()
    os.makedirs(PROF, exist_ok=True)
    stats = os.path.join(OUT, "prof_trace", "trace_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(PROF, f"{a.tag}_kernel_stats.csv"))
    fetch = pmc(os.path.join(OUT, a.pmc_dir), "FETCH_SIZE")
    write = pmc(os.path.join(OUT, a.pmc_dir), "WRITE_SIZE")
    rows, traffic = [], {}
    for k in sorted(set(fetch) | set(write)):
        s = stage(k)
        f, w = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        rows.append({"kernel": k[:90], "stage": s or "", "fetch_bytes": int(f),
                     "write_bytes": int(w), "fetch_x2_bytes": int(2 * f)})
        if s:                                   # a stage may be several kernels: sum them
            t = traffic.setdefault(s, {"hbm_bytes": 0, "fetch_bytes": 0, "write_bytes": 0,
                                       "fetch_x2_bytes": 0, "kernels": [],
                                       "note": "per launch; hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE "
                                               "(MI355X_MICROARCH.md: FETCH_SIZE is half the bytes of "
                                               "16-B/lane streams; 8-B gathers uncalibrated)"})
            t["hbm_bytes"] += int(2 * f + w)                 # guide-corrected (see header)
            t["fetch_bytes"] += int(f)
            t["write_bytes"] += int(w)
            t["fetch_x2_bytes"] += int(2 * f)
            t["kernels"].append(k[:60])
    with open(os.path.join(PROF, f"{a.tag}_pmc.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    json.dump(traffic, open(os.path.join(PROF, "pmc_traffic.json"), "w"), indent=1)
    for r in rows:
        print(r)


if __name__ == "__main__":
    main()
