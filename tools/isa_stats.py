#!/usr/bin/env python3
"""Static instruction counts per kernel of a gfx950 device assembly file.

usage:
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -munsafe-fp-atomics \
        -I include --cuda-device-only -S -o /tmp/raymarch.s \
        segment-anything-nerf_amd/csrc/raymarch.hip
  python tools/isa_stats.py /tmp/raymarch.s [name-filter]

Counts are of the straight-line text (loop bodies once), a proxy for the
VALU issue cost per thread of the march kernels, which are mostly
straight-line per sample.  Also prints the register/LDS/occupancy lines the
compiler emits for each kernel.
"""
import collections
import re
import subprocess
import sys


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    kernels = collections.OrderedDict()
    meta = collections.defaultdict(dict)
    cur = last = None
    for line in open(path):
        t = line.strip()
        if last is not None and t.startswith(";"):
            # the register / occupancy comments follow the kernel's .Lfunc_end
            mm = re.match(r";\s*(NumVgprs|NumAgprs|TotalNumVgprs|ScratchSize|Occupancy|LDSByteSize|NumSgprs):\s*(\S+)", t)
            if mm:
                meta[last][mm.group(1)] = mm.group(2)
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and not line.startswith("\t"):
            cur = m.group(1)
            last = None
            kernels[cur] = collections.Counter()
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            last, cur = cur, None
            continue
        if t.startswith(";"):
            continue
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        c = kernels[cur]
        c["total"] += 1
        if op.startswith("v_mfma"):
            c["mfma"] += 1
        elif op.startswith("v_pk_"):
            c["v_pk"] += 1
            c["valu"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_waitcnt") or op.startswith("s_nop"):
            c["wait"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("global_load") or op.startswith("buffer_load"):
            c["vmem_ld"] += 1
        elif op.startswith("global_store") or op.startswith("buffer_store") or op.startswith("global_atomic"):
            c["vmem_st"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
    names = list(kernels)
    pretty = demangle(names)
    for n, p in zip(names, pretty):
        if filt and filt not in p:
            continue
        c = kernels[n]
        keys = ["total", "valu", "v_pk", "mfma", "salu", "vmem_ld", "vmem_st", "lds"]
        print(p[:90])
        print("   " + " ".join(f"{k}={c[k]}" for k in keys) + "   " +
              " ".join(f"{k}={v}" for k, v in meta[n].items()))


if __name__ == "__main__":
    main()
