#!/usr/bin/env python3
"""SAM-head kernel timing on one MI355X (diagnostic, not the bench line).

Runs samnerf_sam_head_forward on N random head-input rows (the [N, 164] rows
k_final writes) with the default-architecture head (163 -> 256 x 5 +
LayerNorm), times it with HIP events over --iters launches, and checks:
  * every diagnostic variant listed in --variants (SAMNERF_HEAD_V=<v>, read by
    libsamnerf_hip_diag.so only) is bit-identical to the product library;
  * the product head against the exact-fp32 MFMA head (head_mode 1).
usage (GPU box): python tools/head_bench.py [--n 262144] [--variants 0,1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="")
    ap.add_argument("--no-exact", action="store_true")
    a = ap.parse_args()
    from nerf.network import NeRFNetwork
    from samnerf_amd import synth, _lib
    from samnerf_amd.fused import FusedRenderer
    dev = torch.device("cuda", 0)
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=12, prop_log2=10)
    params = synth.make_params(spec, seed=8, emb_scale=0.5, ln_jitter=0.1)
    from nerf.network import default_opt as _do
    opt = _do(with_sam=True, grid_log2=12, s_grid_log2=12, prop_log2=10)
    net = NeRFNetwork(opt)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    net = net.to(dev).eval()
    g = torch.Generator().manual_seed(1)
    rows = torch.randn(a.n, 164, generator=g)
    rows[:, 163] = 0.0
    rows = rows.to(dev)

    def timed(fr):
        out = fr.sam_head(rows)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fr.sam_head(rows)
        e1.record()
        torch.cuda.synchronize()
        return out, e0.elapsed_time(e1) / a.iters

    res = {"n": a.n}
    base, ms = timed(FusedRenderer(net, head_mode=0))
    res["product_ms"] = ms
    if not a.no_exact:
        ex, ms_ex = timed(FusedRenderer(net, head_mode=1))
        res["exact_ms"] = ms_ex
        res["max_abs_vs_exact"] = (base - ex).abs().max().item()
    for v in [s for s in a.variants.split(",") if s]:
        os.environ["SAMNERF_HEAD_V"] = v
        with _lib.diag_library():
            out, ms_v = timed(FusedRenderer(net, head_mode=0))
        res[f"v{v}_ms"] = ms_v
        res[f"v{v}_bit_identical"] = bool(torch.equal(out, base))
        res[f"v{v}_max_abs_diff"] = (out - base).abs().max().item()
    os.environ.pop("SAMNERF_HEAD_V", None)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
