#!/usr/bin/env python3
"""Per-stage counter rates of one view from a tools/pmc_passes.sh output dir.

usage: python tools/pmc_rates.py gpurun_out/pmc_<TAG> > profiles/pmc_rates.json

For each stage of the view (the kernels bench.py's stage events bracket) it
averages every counter over the stage's dispatches and sums the stage's
kernels, per launch of the view (the profiled bench renders the headline
512x512 view, 262,144 rays).  bench.py prices its live stage times with these
(stage_roofline): issued VALU instructions per ray (SQ_INSTS_VALU, priced at
the measured 2.25 cycles per instruction, tools/valu_rate.hip -- round 4 found
SQ_ACTIVE_INST_VALU counting one per simple instruction, not quad-cycles),
MFMA-busy cycles, the wave-cycle shares (SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES), and HBM bytes = 2 x FETCH_SIZE +
WRITE_SIZE (the guide's gfx950 correction).
Every number is recomputable from the table tools/pmc_table.py prints for the
same directory (profiles/<tag>_pmc_table.txt).
"""
import collections
import csv
import glob
import json
import sys

STAGE_KERNELS = {                     # substring of the kernel name -> stage
    "k_get_rays": "prop0", "k_snf": "prop0", "k_prop_sigma<128": "prop0", "k_prop_pdf<128": "prop0",
    "k_prop_sigma<64": "prop1", "k_prop_pdf<64": "prop1",
    "k_final": "final",
    "k_sgrid": "s_grid",
    "k_head_wmax": "sam_head", "k_pack_h16": "sam_head", "k_pack_w8": "sam_head", "k_sam_head": "sam_head",
}
RAYS = 262144


def stage_of(name):
    for k, st in STAGE_KERNELS.items():
        if k in name:
            return st
    return None


def main(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for name, cs in vals.items():
        st = stage_of(name)
        if st is None:
            continue
        d = out.setdefault(st, {"kernels": [], "counters": collections.defaultdict(float)})
        d["kernels"].append(name[:80])
        for c, v in cs.items():
            d["counters"][c] += sum(v) / len(v)          # per dispatch, summed over the stage's kernels
    res = {"rays_per_view": RAYS, "source": root, "stages": {}}
    for st, d in out.items():
        c = d["counters"]
        e = {"kernels": sorted(d["kernels"]), "counters_per_view": dict(c)}
        if "SQ_ACTIVE_INST_VALU" in c:
            e["valu_cycles_per_ray"] = 4.0 * c["SQ_ACTIVE_INST_VALU"] / RAYS
        if "SQ_INSTS_VALU" in c:
            # issued VALU instructions (MFMAs included: they are VALU-encoded; a
            # handful per sample against ~1,000), priced at the measured issue
            # rate of independent VALU streams (profiles/r4_valu_rate.json)
            e["valu_insts_per_ray"] = c["SQ_INSTS_VALU"] / RAYS
        if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
            # wave-cycle shares (MI355X_MICROARCH.md rocprofv3 slots: WAIT_ANY +
            # WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES, disjoint)
            wc = c["SQ_WAVE_CYCLES"]
            e["wave_cycle_shares"] = {"wait_any": c["SQ_WAIT_ANY"] / wc,
                                      "wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                                      "active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc}
        if "SQ_THREAD_CYCLES_VALU" in c:
            # VALU pipe occupancy from the counter (round 6, VERDICT r5 item
            # 2): thread-cycles of VALU execution per SIMD / 64 lanes = the
            # SIMD cycles its VALU spent (full waves), next to the static
            # opcode-mix estimate (valu_insts_per_ray x cycles per instruction)
            e["valu_pipe_cycles_per_ray"] = c["SQ_THREAD_CYCLES_VALU"] / 64.0 / RAYS
        if "SQ_ACTIVE_INST_VALU2" in c:
            e["valu_dual_issue_quad_cycles_per_ray"] = c["SQ_ACTIVE_INST_VALU2"] / RAYS
        if "SQ_VALU_MFMA_COEXEC_CYCLES" in c:
            e["mfma_coexec_cycles_per_ray"] = c["SQ_VALU_MFMA_COEXEC_CYCLES"] / RAYS
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            e["mfma_busy_cycles_per_ray"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / RAYS
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes_per_ray"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0 / RAYS
        if "TA_BUSY_avr" in c and "GRBM_GUI_ACTIVE" in c:
            e["ta_busy_frac_in_pmc_run"] = c["TA_BUSY_avr"] / (c["GRBM_GUI_ACTIVE"] / 8.0)
        res["stages"][st] = e
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
