#!/usr/bin/env python3
"""Per-phase instruction budget of k_final's sample loop.

usage:
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -munsafe-fp-atomics \\
        -I include --cuda-device-only -S -o /tmp/raymarch.s segment-anything-nerf_amd/csrc/raymarch.hip
  python tools/valu_budget.py /tmp/raymarch.s [mangled-kernel-name]

The product kernel's sample loop is straight-line code (LAY 1: the level
classes are compile-time constants), so a static count of its body is the
per-sample-step instruction mix of one wave.  Phases, in program order:
  position  bins -> real bins (IEEE divisions), position, contract, grid scale
  idx0/1    k-block 0 / 1: level descriptors (LDS), cells, fractions, hashed /
            dense corner rows, byte offsets
  ld0/1     the gathers (global_load_dwordx2 / x4) and their hazard s_nops
  sum0/1    corner weights (1 - f, packed products) and the packed corner sums
  mlp       from the first f16 split on: split (v_fma_mix), MFMA, LDS
            fragment reads, boundary (max / ReLU / exponent / permlane)
  composite sigma = exp, alpha, the double cumulative sum, weights, stores
Counts are static instructions per loop trip (divergent branches of the
position counted once), the VALU column is what issues on the VALU pipe, and
`cycles` prices each VALU instruction at its measured issue cost per wave64
at 8 waves per SIMD (profiles/r5v_valu_rate.json, tools/valu_rate.hip):
2.2 cycles for the double-rate fp32 fma / mul / add / sub and integer add /
xor / and / or, 2.5 for v_bitop3, 4.2 for packed fp32 and everything else
4.1, 8.1 for v_fma_mix and the transcendentals.
"""
import collections
import re
import sys

DEFAULT = "_ZN12_GLOBAL__N_17k_finalILi32ELi1ELb0ELb0ELb0ELb0ELi0ELi1ELb0EEEvNS_9FinalArgsE"


def kernel_lines(path, name):
    out, on = [], False
    for line in open(path):
        if line.startswith(name + ":"):
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line.rstrip("\n"))
    return out


def sample_loop(lines):
    """The loop whose body holds the MFMAs: from its header label to the
    backward branch to it."""
    headers = [i for i, l in enumerate(lines) if "Loop Header" in l]
    best = None
    for h in headers:
        lbl = lines[h].split(":")[0]
        for j in range(h + 1, len(lines)):
            t = lines[j].strip()
            if t.startswith(("s_branch", "s_cbranch")) and t.split()[-1] == lbl:
                body = lines[h:j + 1]
                n = sum(1 for x in body if "v_mfma" in x)
                if n and (best is None or n > best[0]):
                    best = (n, body)
    return best[1] if best else []


def ops(body):
    for l in body:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        yield t.split()[0]


FAST = ("v_fma_f32", "v_fmac_f32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_add_u32",
        "v_sub_u32", "v_subrev_u32", "v_xor_b32", "v_and_b32", "v_or_b32")
SLOW = ("v_fma_mix", "v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32", "v_cos_f32")


def cycles(op):
    if op.startswith(SLOW):
        return 8.1
    if op.startswith(FAST):
        return 2.2
    if op.startswith("v_bitop3"):
        return 2.5
    if op.startswith("v_pk_"):
        return 4.2
    return 4.1


def is_gather(op):
    return op in ("global_load_dwordx2", "global_load_dwordx4")


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else DEFAULT
    body = sample_loop(kernel_lines(path, name))
    seq = list(ops(body))
    phases = ["position", "idx0", "ld0", "sum0", "idx1", "ld1", "sum1"]
    ph = 0
    cnt = collections.OrderedDict((p, collections.Counter()) for p in phases + [
        "mlp:split", "mlp:mfma", "mlp:lds", "mlp:boundary", "composite"])
    in_mlp = False
    last_mfma = max(i for i, o in enumerate(seq) if o.startswith("v_mfma"))
    for i, op in enumerate(seq):
        if not in_mlp:
            if op.startswith(("v_fma_mix", "v_cvt_pk_f16_f32")):
                in_mlp = True
            else:
                p = phases[ph]
                if p in ("position", "sum0") and op.startswith("ds_read"):
                    ph += 1
                elif p in ("idx0", "idx1") and is_gather(op):
                    ph += 1
                elif p in ("ld0", "ld1") and not (is_gather(op) or op.startswith(("s_nop", "global_store",
                                                                                    "v_lshl_add_u64",
                                                                                    "s_and_saveexec",
                                                                                    "s_cbranch", "s_or_b64"))):
                    ph += 1
                cnt[phases[min(ph, len(phases) - 1)]][op] += 1
                continue
        if i > last_mfma:
            cnt["composite"][op] += 1
        elif op.startswith(("v_fma_mix", "v_cvt_pk_f16_f32", "v_cvt_f32_f16", "v_mul_f32", "v_sub_f32")):
            cnt["mlp:split"][op] += 1
        elif op.startswith("v_mfma"):
            cnt["mlp:mfma"][op] += 1
        elif op.startswith("ds_"):
            cnt["mlp:lds"][op] += 1
        else:
            cnt["mlp:boundary"][op] += 1
    tot = collections.Counter()
    print(f"{'phase':<14}{'instr':>7}{'VALU':>7}{'cycles':>8}{'VMEM':>6}{'LDS':>5}{'SALU':>6}{'nop':>5}  top opcodes")
    for p, c in cnt.items():
        n = sum(c.values())
        valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
        vmem = sum(v for k, v in c.items() if k.startswith(("global_", "scratch_", "buffer_")))
        lds = sum(v for k, v in c.items() if k.startswith("ds_"))
        salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith(("s_nop", "s_waitcnt")))
        nop = c.get("s_nop", 0)
        cyc = sum(v * cycles(k) for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
        tot.update({"instr": n, "valu": valu, "vmem": vmem, "lds": lds, "salu": salu, "nop": nop, "cyc": cyc})
        top = ", ".join(f"{k} {v}" for k, v in c.most_common(4))
        print(f"{p:<14}{n:>7}{valu:>7}{cyc:>8.0f}{vmem:>6}{lds:>5}{salu:>6}{nop:>5}  {top}")
    print(f"{'total':<14}{tot['instr']:>7}{tot['valu']:>7}{tot['cyc']:>8.0f}{tot['vmem']:>6}{tot['lds']:>5}"
          f"{tot['salu']:>6}{tot['nop']:>5}")


if __name__ == "__main__":
    main()
