#!/usr/bin/env python3
"""Build libsamnerf_hip.so (gfx950) in-tree with hipcc.

The library is the C ABI of include/samnerf_hip.h.  Flags:
  --offload-arch=gfx950   MI355X only (no multi-arch / CUDA paths)
  -ffp-contract=off       every FMA is explicit (__builtin_fmaf) so device
                          arithmetic reproduces the reference's op order
  -munsafe-fp-atomics     float atomicAdd -> global_atomic_add_f32 (no CAS loop)
usage: python segment-anything-nerf_amd/build.py [--jobs N]
"""
import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "samnerf_amd")
LIB = os.path.join(OUT_DIR, "libsamnerf_hip.so")
OBJ_DIR = os.path.join(HERE, "build", "obj")
# the diagnostic build: the same sources with the kernels' A/B variant switches
# read from the environment (samnerf_common.h diag_env), for the bit-identity
# tests of the alternative forms; never loaded by the product path
DIAG_LIB = os.path.join(OUT_DIR, "libsamnerf_hip_diag.so")
DIAG_OBJ_DIR = os.path.join(HERE, "build", "obj_diag")

SOURCES = ["common.cpp", "grid_encoder.hip", "sh_freq_encoder.hip", "raymarch.hip",
           "sam_head.hip", "tile_codec.hip", "train_optim.hip", "sam_head_train.hip",
           "mask_head.hip", "rgb_train.hip", "mask_head_train.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-munsafe-fp-atomics", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
         "-I", os.path.join(HERE, "..", "include")]


def _newer(src, obj):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    deps.append(os.path.join(HERE, "..", "include", "samnerf_hip.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, diag=False):
    obj = os.path.join(DIAG_OBJ_DIR if diag else OBJ_DIR, src + ".o")
    path = os.path.join(CSRC, src)
    if not _newer(path, obj):
        return obj
    flags = FLAGS + (["-DSAMNERF_DIAG_VARIANTS"] if diag else [])
    cmd = [HIPCC] + flags + ["-c", path, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-x", "hip"] + flags + ["-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
    return obj


def _link(objs, lib):
    if not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")


ASM_DIR = os.path.join(HERE, "build", "asm")


def build_asm(jobs=None, sources=None):
    """Device assembly (hipcc --cuda-device-only -S, the product flags) of
    every product source into build/asm/<src>.s, rebuilt when older than its
    inputs: the input of the inline-asm hazard lint (tools/isa_hazards.py,
    tests/test_isa_hazards.py), which needs the ;;#ASMSTART / ;;#ASMEND
    markers a disassembly does not carry."""
    os.makedirs(ASM_DIR, exist_ok=True)
    srcs = [s for s in (sources or SOURCES) if s.endswith(".hip")]

    def one(src):
        out = os.path.join(ASM_DIR, src + ".s")
        if _newer(os.path.join(CSRC, src), out):
            cmd = [HIPCC] + FLAGS + ["--cuda-device-only", "-S", os.path.join(CSRC, src), "-o", out]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc -S failed on {src}:\n{r.stderr}")
        return out

    with cf.ThreadPoolExecutor(jobs or min(len(srcs), os.cpu_count() or 4, 8)) as ex:
        return list(ex.map(one, srcs))


def build(jobs=None, verbose=True, diag=True):
    """The product library, and (diag=True) the diagnostic build beside it."""
    os.makedirs(OBJ_DIR, exist_ok=True)
    os.makedirs(DIAG_OBJ_DIR, exist_ok=True)
    jobs = jobs or min(2 * len(SOURCES), os.cpu_count() or 4, 8)
    work = [(src, False) for src in SOURCES] + ([(src, True) for src in SOURCES] if diag else [])
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda a: _compile(*a), work))
    _link(objs[:len(SOURCES)], LIB)
    if diag:
        _link(objs[len(SOURCES):], DIAG_LIB)
    if verbose:
        print(f"[samnerf] built {LIB}" + (f" and {os.path.basename(DIAG_LIB)}" if diag else ""))
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args()
    try:
        build(a.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
