#!/usr/bin/env python3
"""Static MFMA / VALU / memory hazard lint for gfx950 machine code
(VERDICT r5 item 3).

Input: a shared library built by segment-anything-nerf_amd/build.py (its
.hip_fatbin section is split into the clang offload bundles of each
translation unit, the gfx950 code objects are disassembled with
llvm-objdump), or a device assembly file (hipcc --cuda-device-only -S).
Every kernel is walked in program order; wait states are counted as the
hardware counts them: one per issued instruction, N + 1 for `s_nop N`.

Rules (the pairs hipcc pads for its own code -- LLVM GCNHazardRecognizer's
gfx940/gfx950 MAI hazards, cdna_hip_programming.md 5.7 -- and that an
`asm volatile` string must pad itself, because nothing inside one is padded):
  R1  a VALU write of a VGPR, then an MFMA reading it as SrcA / SrcB / SrcC:
      2 wait states;
  R2  an MFMA of P passes writing its D registers, then any non-MFMA
      instruction reading or writing them (VALU, VMEM, LDS), or an MFMA
      reading them as SrcA / SrcB: P + 4 for an XDL op (f16 / bf16 / 8-bit;
      the guide's 12 for an 8-pass XDL on gfx950), P + 2 for the f32 ones;
      the next MFMA taking D whole as its SrcC (an accumulation chain) needs
      none;
  R3  an MFMA reading SrcC, then a non-MFMA instruction writing any of those
      registers (write-after-read while the MFMA still reads C): P - 1.
Report only (not a failure; the hypothesis of VERDICT r5 item 3 for the
removed k_final prefetch form):
  R4  a VMEM or LDS load issued within 4 P wait states of an MFMA (the cycles
      it may still execute, one instruction at least one cycle) whose
      destination overlaps that MFMA's SrcA / SrcB / SrcC -- the load may
      land while the MFMA still reads.  LLVM guards only SrcC (R3); R4 adds
      A / B.

Which pairs count: in a device assembly file (.s) only the pairs with the
producer or the consumer inside an inline-asm statement (;;#ASMSTART ..
;;#ASMEND) -- hipcc pads its own instructions with its hazard model and does
not pad asm -- unless --all; a disassembled library has no asm markers, so
there every pair is reported (the compiler's own 16x16x32 chains then show
as R2 / R3 pairs that LLVM does not pad: its model for those shapes is
looser than the table above, which is meant for asm).

Control flow: straight-line order, plus each loop's back edge (the last 48
instructions before a backward branch followed by the first 48 after its
target).  Passes per MFMA from its shape: M N K 2 / (1024 flops per cycle
for f16 / bf16, 2048 for 8-bit, 64 for f32) / 4 cycles per pass.

usage: python tools/isa_hazards.py LIB.so|FILE.s [--kernel SUBSTR] [--verbose]
"""
import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
REG = re.compile(r"^(v|a)(?:\[(\d+):(\d+)\]|(\d+))$")


def code_objects(lib):
    """The gfx950 code objects of every offload bundle in lib's .hip_fatbin."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
        data = open(fb, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for s in starts:
        n = struct.unpack_from("<Q", data, s + 24)[0]
        p = s + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                out.append(data[s + off:s + off + size])
    return out


def disassemble(blob):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(blob)
        f.flush()
        r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn",
                            "--no-leading-addr", f.name], capture_output=True, text=True, check=True)
    return r.stdout


def functions_from_objdump(text):
    funcs, name, body = {}, None, []
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+ )?<(\S+)>:\s*$", line)
        if m:
            if name:
                funcs[name] = body
            name, body = m.group(2), []
            continue
        if name is not None:
            body.append(line)
    if name:
        funcs[name] = body
    return funcs


def functions_from_asm(text):
    funcs, name, body = {}, None, []
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name, body = m.group(1), []
            continue
        if name is None:
            continue
        if line.startswith(".Lfunc_end"):
            funcs[name] = body
            name = None
            continue
        body.append(line)
    return funcs


class Inst:
    __slots__ = ("op", "ops", "text", "label", "target", "weight", "asm")

    def __init__(self, op, ops, text, label=None, target=None, weight=1, asm=False):
        self.op, self.ops, self.text, self.label, self.target, self.weight = op, ops, text, label, target, weight
        self.asm = asm


def parse(body):
    """Instructions (with labels attached to the next one) of one function;
    asm = inside an inline-asm statement (.s input)."""
    insts, pending, in_asm = [], None, False
    for raw in body:
        if ";;#ASMSTART" in raw:
            in_asm = True
            continue
        if ";;#ASMEND" in raw:
            in_asm = False
            continue
        line = raw.split("//")[0].split(";")[0].strip()
        if not line or line.startswith("."):
            m = re.match(r"^(\.L\w+):", line)
            if m:
                pending = m.group(1)
            continue
        m = re.match(r"^<?([\w.$]+)>?:$", line)
        if m:
            pending = m.group(1)
            continue
        parts = line.split(None, 1)
        op = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        w = 1
        if op == "s_nop":
            try:
                w = int(ops[0], 0) + 1
            except (ValueError, IndexError):
                w = 1
        tgt = None
        if op.startswith(("s_branch", "s_cbranch")) and ops:
            t = ops[-1].split()[0].strip("<>")
            tgt = t.split("+")[0]
        insts.append(Inst(op, ops, line, pending, tgt, w, in_asm))
        pending = None
    return insts


def regs(tok):
    tok = tok.strip().split()[0] if tok.strip() else ""
    m = REG.match(tok)
    if not m:
        return frozenset()
    f = m.group(1)
    if m.group(4) is not None:
        return frozenset({(f, int(m.group(4)))})
    return frozenset((f, i) for i in range(int(m.group(2)), int(m.group(3)) + 1))


def mfma_passes(op):
    m = re.search(r"(\d+)x(\d+)x(\d+)", op)
    if not m:
        return 8
    M, N, K = (int(x) for x in m.groups())
    if "f32_" in op and op.rstrip("_e64").endswith(("f32", "xf32")) and "f16" not in op and "bf16" not in op:
        rate = 64
    elif re.search(r"(fp8|bf8|i8|f8f6f4)", op):
        rate = 2048
    else:
        rate = 1024
    cyc = M * N * K * 2 / rate
    return max(1, int(round(cyc / 4)))


def is_xdl(op):
    return not re.search(r"_f32_\d+x\d+x\d+_?(f32|xf32)|_f64_", op)


def d_after(op, P):
    return P + 4 if is_xdl(op) else P + 2


def is_mfma(op):
    return op.startswith(("v_mfma", "v_smfmac"))


def defs_uses(ins):
    """(defs, uses) VGPR / AGPR sets of one instruction."""
    op, ops = ins.op, ins.ops
    if not ops:
        return frozenset(), frozenset()
    allr = [regs(o) for o in ops]
    if is_mfma(op):
        return allr[0], frozenset().union(*allr[1:4]) if len(allr) > 1 else frozenset()
    if op.startswith("v_"):
        if op.startswith(("v_cmp_", "v_readfirstlane", "v_readlane")) and not op.startswith("v_cmpx"):
            return frozenset(), frozenset().union(*allr)
        if op.startswith(("v_permlane", "v_swap")):
            d = allr[0] | (allr[1] if len(allr) > 1 else frozenset())
            return d, d
        return allr[0], frozenset().union(*allr[1:]) if len(allr) > 1 else frozenset()
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        if "_lds" in op or "store" in op or "_wb" in op or "_inv" in op:
            return frozenset(), frozenset().union(*allr)
        if "atomic" in op and not re.search(r"\b(sc0|glc)\b", ins.text):
            return frozenset(), frozenset().union(*allr)
        return allr[0], frozenset().union(*allr[1:]) if len(allr) > 1 else frozenset()
    if op.startswith("ds_"):
        if op.startswith(("ds_write", "ds_store")) or (op.startswith("ds_") and "_rtn" not in op and
                                                        op.startswith(("ds_add", "ds_max", "ds_min",
                                                                       "ds_and", "ds_or", "ds_xor"))):
            return frozenset(), frozenset().union(*allr)
        return allr[0], frozenset().union(*allr[1:]) if len(allr) > 1 else frozenset()
    return frozenset(), frozenset()


def is_load(ins):
    op = ins.op
    return (op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load", "ds_read", "ds_load"))
            and "_lds" not in op)


def check_seq(seq, found, where, asm_only=False):
    """Walk one instruction sequence; append (rule, need, have, producer,
    consumer, where) to found (asm_only: pairs touching an asm statement)."""
    n0 = len(found)
    pos, p = [], 0
    for ins in seq:
        pos.append(p)
        p += ins.weight
    du = [defs_uses(i) for i in seq]
    recent_valu = []      # (index, defs)
    recent_mfma = []      # (index, passes, D, A|B, C, D-hazard wait states)
    for j, ins in enumerate(seq):
        d, u = du[j]
        op = ins.op
        # expire producers beyond every rule's reach
        recent_valu = [(i, dd) for i, dd in recent_valu if pos[j] - pos[i] - 1 < 2]
        recent_mfma = [t for t in recent_mfma if pos[j] - pos[t[0]] - 1 < max(4 * t[1], t[1] + 4)]
        if is_mfma(op):
            a_b = frozenset().union(*(regs(o) for o in ins.ops[1:3]))
            c = regs(ins.ops[3]) if len(ins.ops) > 3 else frozenset()
            for i, dd in recent_valu:
                if dd & (a_b | c):
                    found.append(("R1", 2, pos[j] - pos[i] - 1, seq[i].text, ins.text, where))
            for i, P, D, AB, C, R in recent_mfma:
                ws = pos[j] - pos[i] - 1
                if D & a_b and ws < R:
                    found.append(("R2", R, ws, seq[i].text, ins.text, where))
                if D & c and c != D and ws < R - 1:
                    found.append(("R2", R - 1, ws, seq[i].text, ins.text, where))
            P = mfma_passes(op)
            # the last writer of a register is the one a later reader waits for
            recent_mfma = [(i, P0, D - d, AB, C, R) for i, P0, D, AB, C, R in recent_mfma]
            recent_valu = [(i, dd - d) for i, dd in recent_valu]
            recent_mfma.append((j, P, d, a_b, c, d_after(op, P)))
            continue
        if d or u:
            for i, P, D, AB, C, R in recent_mfma:
                ws = pos[j] - pos[i] - 1
                if D & (d | u) and ws < R:
                    found.append(("R2", R, ws, seq[i].text, ins.text, where))
                if C & d and not (C == D) and ws < P - 1:
                    found.append(("R3", P - 1, ws, seq[i].text, ins.text, where))
                if is_load(ins) and (AB | C) & d and ws < 4 * P:
                    found.append(("R4", 4 * P, ws, seq[i].text, ins.text, where))
        if d:
            recent_mfma = [(i, P0, D - d, AB, C, R) for i, P0, D, AB, C, R in recent_mfma]
            recent_valu = [(i, dd - d) for i, dd in recent_valu]
        if op.startswith("v_") and d:
            recent_valu.append((j, d))
    if asm_only:
        idx = {id(x): k for k, x in enumerate(seq)}
        asm_text = {seq[k].text for k in range(len(seq)) if seq[k].asm}
        keep = [f for f in found[n0:] if f[3] in asm_text or f[4] in asm_text]
        del found[n0:]
        found.extend(keep)


def lint(insts, name, found, asm_only=False):
    check_seq(insts, found, name, asm_only)
    labels = {ins.label: k for k, ins in enumerate(insts) if ins.label}
    for b, ins in enumerate(insts):
        if ins.target in labels and labels[ins.target] <= b:
            l = labels[ins.target]
            wrap = insts[max(l, b - 48):b + 1] + insts[l:min(l + 48, b + 1)]
            n0 = len(found)
            check_seq(wrap, found, name + " (loop wrap)", asm_only)
            # keep only pairs that cross the back edge
            keep = [f for f in found[n0:] if f[2] >= 0]
            del found[n0:]
            seen = {(f[0], f[3], f[4]) for f in found}
            found.extend(f for f in keep if (f[0], f[3], f[4]) not in seen)


def demangle(names):
    try:
        r = subprocess.run([os.path.join(LLVM, "llvm-cxxfilt")], input="\n".join(names), capture_output=True,
                           text=True)
        return r.stdout.splitlines()
    except OSError:
        return names


def run(path, kernel=None, all_pairs=False):
    """{kernel: [(rule, need, have, producer, consumer, where)]} for every
    kernel of `path` (a .so or a .s) whose name contains `kernel`."""
    asm_only = False
    if path.endswith(".s"):
        funcs = functions_from_asm(open(path).read())
        asm_only = not all_pairs
    else:
        funcs = {}
        for blob in code_objects(path):
            funcs.update(functions_from_objdump(disassemble(blob)))
    res = {}
    for name, body in funcs.items():
        if kernel and kernel not in name:
            continue
        found = []
        lint(parse(body), name, found, asm_only)
        res[name] = found
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--all", action="store_true", help=".s input: every pair, not only asm-touching ones")
    a = ap.parse_args()
    res = run(a.path, a.kernel, a.all)
    names = list(res)
    pretty = dict(zip(names, demangle(names)))
    tot = {"R1": 0, "R2": 0, "R3": 0, "R4": 0}
    for name, found in res.items():
        if not found:
            continue
        by = {}
        for f in found:
            by.setdefault(f[0], []).append(f)
            tot[f[0]] += 1
        print(f"{pretty[name][:110]}: " + ", ".join(f"{r} {len(v)}" for r, v in sorted(by.items())))
        if a.verbose:
            for f in found:
                print(f"   {f[0]} need {f[1]} have {f[2]}: {f[3]}  ->  {f[4]}")
    print(f"kernels {len(res)}; violations R1 {tot['R1']} R2 {tot['R2']} R3 {tot['R3']}; R4 (report) {tot['R4']}")
    return 1 if tot["R1"] + tot["R2"] + tot["R3"] else 0


if __name__ == "__main__":
    sys.exit(main())
