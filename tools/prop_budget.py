#!/usr/bin/env python3
"""Per-phase VALU budget of the proposal sigma kernels:
k_prop_sigma<128, DDDHH> and <64, DDHHH> are one (ray, sample) per thread,
straight-line apart from the uniform-dense / per-lane branch of each level,
so a static count of the kernel is one wave-sample's instruction mix.  The
phases are assigned by opcode and operand class, not by program order (the
scheduler interleaves them):

  record     the ray record / bins loads and their 64-bit / byte addresses
  bins       real_bin (spacing_inv: IEEE division), the midpoint, the
             position o + t d and the L-inf contraction
  locate     per level and axis: grid scale, fma, med3 clamp, cvt, fract
  rows       corner rows: hashed XOR terms, dense sums, shifts, selects
  gather     the corner loads (global / scalar)
  trilinear  corner weights (1 - f, products) and the weighted corner sums
  mlp        the 10 -> 16 -> 1 MLP on packed fp32 (SGPR weights) and ReLU
  out        trunc_exp (v_exp), delta * sigma, the store

Cycles price each VALU instruction at its measured issue cost per wave64
(profiles/r5v_valu_rate.json, tools/valu_budget.py): 2.2 for fp32 fma / mul
/ add and integer add / xor / and / or, 2.5 v_bitop3, 4.2 packed fp32, 8.1
v_exp / v_rcp / v_fma_mix, 4.1 the rest.

usage:
  python tools/prop_budget.py segment-anything-nerf_amd/build/asm/raymarch.hip.s
(build.py build_asm writes that file; tests/test_isa_hazards.py builds it)"""
import collections
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from valu_budget import cycles, kernel_lines  # noqa: E402

KERNELS = {
    "k_prop_sigma<128, DDDHH>": "_ZN12_GLOBAL__N_112k_prop_sigmaILi128ELb1ELi0ELj7ELj24EEEvNS_8PropArgsE",
    "k_prop_sigma<64, DDHHH>": "_ZN12_GLOBAL__N_112k_prop_sigmaILi64ELb0ELi0ELj3ELj28EEEvNS_8PropArgsE",
}
PHASES = ["record", "bins", "locate", "rows", "gather", "trilinear", "mlp", "out"]


def classify(op, line, state):
    """Phase of one instruction; `state` tracks whether the MLP has begun
    (the first packed fma with an SGPR weight pair after the gathers)."""
    if op.startswith(("global_load", "s_load", "s_buffer_load", "buffer_load")):
        return "gather" if state["gathers"] else "record"
    if op.startswith("global_store"):
        return "out"
    if op.startswith(("v_exp_f32", "v_ldexp", "v_frexp")):
        return "out"
    if op.startswith(("v_div_", "v_rcp_f32")) or (op.startswith("v_cndmask") and not state["gathers"]):
        return "bins"
    if op.startswith(("v_med3_f32", "v_fract_f32", "v_cvt_u32_f32", "v_cvt_i32_f32", "v_floor")):
        state["gathers"] = True
        return "locate"
    if op.startswith(("v_xor_b32", "v_bitop3", "v_and_b32", "v_or_b32", "v_lshl", "v_add_lshl", "v_lshl_add",
                      "v_mul_u32_u24", "v_mul_lo_u32", "v_mad_u32_u24", "v_min_u32", "v_max_u32", "v_add_u32",
                      "v_sub_u32", "v_add3_u32", "v_readfirstlane", "v_cmp_eq_u32", "v_cmp_lt_u32")):
        return "rows" if state["gathers"] else "record"
    if op.startswith(("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32")):
        if state["mlp"] or re.search(r"s\[\d+:\d+\]", line):
            state["mlp"] = True
            return "mlp"
        return "trilinear" if state["gathers"] else "bins"
    if op.startswith(("v_max_f32", "v_max_i32")) and state["mlp"]:
        return "mlp"
    if op.startswith(("v_fma_f32", "v_fmac_f32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32")):
        if state["mlp"]:
            return "mlp"
        return "trilinear" if state["gathers"] else "bins"
    if not state["gathers"]:
        return "bins"
    return "mlp" if state["mlp"] else "trilinear"


def budget(lines):
    cnt = collections.OrderedDict((p, collections.Counter()) for p in PHASES)
    state = {"gathers": False, "mlp": False}
    for l in lines:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith(("s_waitcnt", "s_nop", "s_endpgm", "s_cbranch", "s_branch", "s_and_saveexec",
                          "s_or_b64", "s_mov_b64", "s_andn2", "s_xor_b64")):
            continue
        cnt[classify(op, t, state)][op] += 1
    return cnt


def main():
    path = sys.argv[1]
    for title, name in KERNELS.items():
        lines = kernel_lines(path, name)
        if not lines:
            print(title, "not found")
            continue
        cnt = budget(lines)
        print(f"== {title}  (static, one wave-sample)")
        print(f"{'phase':<11}{'instr':>7}{'VALU':>7}{'cycles':>8}{'VMEM':>6}{'SMEM':>6}  top opcodes")
        tot = [0, 0, 0.0, 0, 0]
        for p, c in cnt.items():
            n = sum(c.values())
            valu = sum(v for k, v in c.items() if k.startswith("v_"))
            cyc = sum(v * cycles(k) for k, v in c.items() if k.startswith("v_"))
            vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_")))
            smem = sum(v for k, v in c.items() if k.startswith("s_load"))
            top = ", ".join(f"{k} {v}" for k, v in c.most_common(4))
            print(f"{p:<11}{n:>7}{valu:>7}{cyc:>8.0f}{vmem:>6}{smem:>6}  {top}")
            for i, x in enumerate((n, valu, cyc, vmem, smem)):
                tot[i] += x
        print(f"{'total':<11}{tot[0]:>7}{tot[1]:>7}{tot[2]:>8.0f}{tot[3]:>6}{tot[4]:>6}")


if __name__ == "__main__":
    main()
