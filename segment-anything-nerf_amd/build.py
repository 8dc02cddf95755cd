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

SOURCES = ["common.cpp", "grid_encoder.hip", "sh_freq_encoder.hip", "raymarch.hip",
           "sam_head.hip", "tile_codec.hip", "train_optim.hip", "sam_head_train.hip",
           "mask_head.hip", "rgb_train.hip"]
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


def _compile(src):
    obj = os.path.join(OBJ_DIR, src + ".o")
    path = os.path.join(CSRC, src)
    if not _newer(path, obj):
        return obj
    cmd = [HIPCC] + FLAGS + ["-c", path, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-x", "hip"] + FLAGS + ["-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
    return obj


def build(jobs=None, verbose=True):
    os.makedirs(OBJ_DIR, exist_ok=True)
    jobs = jobs or min(len(SOURCES), os.cpu_count() or 4, 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"[samnerf] built {LIB}")
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
