#!/usr/bin/env python3
"""Kernel-trace driver for the training side lines (run under rocprofv3
--kernel-trace --stats): `--what cfg5` runs bench.train_steps (the
distillation step), `--what mask` bench.mask_train_steps (the --with_mask
step, HIP kernels), each for --steps steps after --warmup."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["cfg5", "mask"], default="cfg5")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--deterministic", action="store_true")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    if a.what == "cfg5":
        r = bench.train_steps(dev, a.steps, a.warmup, deterministic=a.deterministic)
    else:
        r = bench.mask_train_steps(dev, a.steps, a.warmup, fused=True)
    print(a.what, r)


if __name__ == "__main__":
    main()
