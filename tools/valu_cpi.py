#!/usr/bin/env python3
"""Issue cycles per VALU instruction of each stage's product kernel, from its
ISA and the measured per-opcode rates (profiles/r5v_valu_rate.json, 8 waves
per SIMD).  bench.py's VALU roofline multiplies the PMC-counted VALU
instructions (SQ_INSTS_VALU) by this figure instead of the v_fma_f32 rate
for every instruction: gfx950 issues v_fma / v_mul / v_add in ~2.2 cycles
per wave64 instruction but conversions, max / min / med3, fract, shifts with
adds, mul_lo and the packed fp32 ops in ~4.1-4.2 and v_fma_mix / exp in ~8.1.

The mix is the static one of the kernel's hot region: the loop holding the
most VALU instructions (k_final's sample loop), or the whole body (the
loop-free proposal kernels; k_sgrid_box4 and the SAM head, whose rotated loops
hold nearly all of it).  Writes
profiles/r6_valu_cpi.json.  usage (CPU, from the repo root):
  python tools/valu_cpi.py
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "segment-anything-nerf_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-munsafe-fp-atomics",
         "-I", os.path.join(ROOT, "include"), "--cuda-device-only", "-S"]
STAGES = {
    "prop0": ("raymarch.hip", "_ZN12_GLOBAL__N_112k_prop_sigmaILi128ELb1ELi0ELj7ELj24EEEvNS_8PropArgsE"),
    "prop1": ("raymarch.hip", "_ZN12_GLOBAL__N_112k_prop_sigmaILi64ELb0ELi0ELj3ELj28EEEvNS_8PropArgsE"),
    "final": ("raymarch.hip", "_ZN12_GLOBAL__N_17k_finalILi32ELi1ELb0ELb0ELb0ELb0ELi0ELi1ELb0EEEvNS_9FinalArgsE"),
    "s_grid": ("raymarch.hip", "_ZN12_GLOBAL__N_112k_sgrid_box4ILi32ELb0EEEvNS_9SgridArgsE"),
    "sam_head": ("sam_head.hip", None),     # the product head: k_sam_head_w8<4, 8, true> (round 6)
}
FAST = ("v_fma_f32", "v_fmac_f32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_add_u32",
        "v_sub_u32", "v_subrev_u32", "v_xor_b32", "v_and_b32", "v_or_b32")
SLOW = ("v_fma_mix", "v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32", "v_cos_f32")


def rate_table():
    d = json.load(open(os.path.join(ROOT, "profiles", "r5v_valu_rate.json")))["kinds"]
    return {k: v["8"]["cycles_per_inst"] for k, v in d.items()}


def cycles(op, rates):
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    if base.startswith(SLOW):
        return rates.get("v_fma_mixlo_f16", 8.1)
    if base in rates and not base.startswith("v_cndmask"):
        return rates[base]
    if base.startswith(FAST):
        return rates.get("v_fma_f32", 2.2)
    if base.startswith("v_bitop3"):
        return rates.get("v_bitop3_b32", 2.5)
    if base.startswith("v_pk_"):
        return rates.get("v_pk_fma_f32", 4.2)
    return rates.get("v_max_i32", 4.1)


def kernel_body(asm, name):
    out, on = [], False
    for line in asm.splitlines():
        if line.startswith(name + ":"):
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line)
    return out


def ops(lines):
    for l in lines:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        yield t.split()[0]


def is_valu(op):
    return op.startswith("v_") and not op.startswith("v_mfma")


def hot_region(body):
    """The loop (header label .. its backward branch) with the most VALU
    instructions, else the whole body."""
    best = None
    for i, l in enumerate(body):
        if "Loop Header" not in l:
            continue
        lbl = l.split(":")[0]
        for j in range(i + 1, len(body)):
            t = body[j].strip()
            if t.startswith(("s_branch", "s_cbranch")) and t.split()[-1] == lbl:
                n = sum(1 for o in ops(body[i:j + 1]) if is_valu(o))
                if best is None or n > best[0]:
                    best = (n, body[i:j + 1], "loop")
    total = sum(1 for o in ops(body) if is_valu(o))
    # a rotated loop (latch placed before its header: the SAM head's tile
    # loop, k_sgrid_box4's sample loop) is not found this way; then the whole
    # body, whose prologue is small next to the unrolled loop
    if best is None or best[0] < 0.2 * total:
        return body, "body"
    return best[1], best[2]


def main():
    rates = rate_table()
    asm = {}
    for f in sorted({v[0] for v in STAGES.values()}):
        out = subprocess.run(["hipcc", *FLAGS, "-o", "-", os.path.join(SRC, f)], check=True,
                             capture_output=True, text=True).stdout
        asm[f] = out
    res = {"what": "issue cycles per VALU instruction of each stage's hot region (static opcode mix x "
                   "profiles/r5v_valu_rate.json at 8 waves per SIMD; tools/valu_cpi.py)", "stages": {}}
    for st, (f, name) in STAGES.items():
        if name is None:
            name = next(m for m in re.findall(r"^(\S*k_sam_head_w8\S*):", asm[f], re.M)
                        if "ILi4ELi8ELb1E" in m)
        region, kind = hot_region(kernel_body(asm[f], name))
        v = [o for o in ops(region) if is_valu(o)]
        cyc = sum(cycles(o, rates) for o in v)
        res["stages"][st] = {"kernel": name, "region": kind, "valu_insts": len(v), "valu_cycles": round(cyc, 1),
                             "cycles_per_inst": round(cyc / max(1, len(v)), 3)}
        print(st, res["stages"][st]["region"], len(v), round(cyc / max(1, len(v)), 3), file=sys.stderr)
    json.dump(res, open(os.path.join(ROOT, "profiles", "r6_valu_cpi.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
