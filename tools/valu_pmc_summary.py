#!/usr/bin/env python3
"""Per-dispatch summary of tools/valu_rate.hip under rocprofv3 --pmc
(tools/prof_r4.sh): for each instruction kind and grid (resident waves per
SIMD = grid / (256 CUs x 4 SIMDs x 64 lanes)), the counters averaged over the
run's dispatches and the VALU instructions issued per SIMD-cycle,
SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) -- the same basis
bench.py's roofline applies to the march kernels.
usage: python tools/valu_pmc_summary.py gpurun_out/prof_<tag>/valu_pmc > profiles/r4_valu_rate_pmc.txt"""
import collections
import csv
import glob
import sys

KINDS = {"k_valu<0>": "v_fma_f32", "k_valu<1>": "v_pk_fma_f32", "k_valu<2>": "v_exp_f32",
         "k_valu<3>": "v_xor_b32+v_add_u32"}
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = next((v for n, v in KINDS.items() if n in r["Kernel_Name"]), None)
        if k:
            vals[(k, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("kind waves/SIMD SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE insts/SIMD-cycle active/insts")
for (k, g), cs in sorted(vals.items()):
    c = {n: sum(v) / len(v) for n, v in cs.items()}
    waves = g / (256 * 4 * 64)
    simd_cyc = c["GRBM_GUI_ACTIVE"] / 8.0 * 1024
    print(f"{k} {waves:g} {c['SQ_INSTS_VALU']:.4g} {c['SQ_ACTIVE_INST_VALU']:.4g} {c['GRBM_GUI_ACTIVE']:.4g} "
          f"{c['SQ_INSTS_VALU'] / simd_cyc:.3f} {c['SQ_ACTIVE_INST_VALU'] / c['SQ_INSTS_VALU']:.3f}")
