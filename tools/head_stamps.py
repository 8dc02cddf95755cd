#!/usr/bin/env python3
"""Where a SAM-head wave's cycles go (diagnostic form 13 of k_sam_head_h16,
libsamnerf_hip_diag.so; form 21 = the persistent k_sam_head_h16q, clock
only): s_memtime marks at the phase boundaries of every
wave, averaged over the waves of a 262,144-row launch.

Phases: prologue (bias / x loads, stream primed), the steps of each layer
(per step: cycles / k-blocks), each layer boundary (bias, leaky_relu, max,
hi/lo split), the LayerNorm sums; plus the kernel span and the gap between
consecutive blocks on a CU (HW_ID).  usage (GPU box): python tools/head_stamps.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))

PHASES = [("prologue", 0, 1, 1), ("L0 steps", 1, 2, 11), ("L0 boundary", 2, 3, 1),
          ("L1 steps", 3, 4, 16), ("L1 boundary + x reload", 4, 5, 1), ("L2 steps", 5, 6, 27),
          ("L2 boundary", 6, 7, 1), ("L3 steps", 7, 8, 16), ("L3 boundary", 8, 9, 1),
          ("L4 steps", 9, 10, 16), ("L4 finish", 10, 11, 1), ("LayerNorm sums", 11, 12, 1)]


def main():
    from nerf.network import NeRFNetwork, default_opt
    from samnerf_amd import synth, _lib
    from samnerf_amd.fused import FusedRenderer
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    form = sys.argv[2] if len(sys.argv) > 2 else "13"      # 21: the persistent form (clock only)
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=12, prop_log2=10)
    params = synth.make_params(spec, seed=8, emb_scale=0.5, ln_jitter=0.1)
    net = NeRFNetwork(default_opt(with_sam=True, grid_log2=12, s_grid_log2=12, prop_log2=10))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    net = net.to(dev).eval()
    rows = torch.randn(n, 164, generator=torch.Generator().manual_seed(1))
    rows[:, 163] = 0.0
    rows = rows.to(dev)
    blocks = (n + 127) // 128
    st = torch.zeros(blocks * 4 * 16, dtype=torch.int64, device=dev)
    base = FusedRenderer(net, head_mode=0).sam_head(rows)
    os.environ["SAMNERF_HEAD_V"] = form
    os.environ["SAMNERF_HEAD_STAMPS"] = "%x" % st.data_ptr()
    with _lib.diag_library():
        fr = FusedRenderer(net, head_mode=0)
        for _ in range(3):
            out = fr.sam_head(rows)
        torch.cuda.synchronize()
    os.environ.pop("SAMNERF_HEAD_V")
    os.environ.pop("SAMNERF_HEAD_STAMPS")
    t = st.view(blocks, 4, 16).cpu().numpy().astype(np.int64)       # form 21: rows of the first workgroups only
    res = {"n": n, "bit_identical": bool(torch.equal(out, base))}
    wave = t[:, :, 12] - t[:, :, 0]
    res["wave_cycles_mean"] = float(wave.mean())
    # shader clock over the wave's life: s_memtime ticks / (s_memrealtime ticks / 100 MHz)
    res["clock_ghz_mean"] = float((wave / np.maximum(t[:, :, 13], 1)).mean() * 0.1)
    if form == "21":                                       # marks 0 and 12 only, one per workgroup life
        live = t[:, 0, 13] > 0
        w = t[live][:, :, 12].astype(np.float64)
        res = {"n": n, "form": 21, "bit_identical": res["bit_identical"],
               "clock_ghz_mean": float((w / t[live][:, :, 13]).mean() * 0.1),
               "wave_cycles_mean": float(w.mean()), "workgroups": int(live.sum())}
        print(json.dumps(res, indent=1))
        return
    res["phases"] = {}
    for name, i, j, k in PHASES:
        d = (t[:, :, j] - t[:, :, i]).astype(np.float64)
        res["phases"][name] = {"cycles": round(float(d.mean())), "per_kblock": round(float(d.mean()) / k),
                               "frac": round(float(d.mean() / wave.mean()), 4)}
    # block-level: span, skew between the block's 4 waves, gaps on a CU
    res["wave_start_skew_mean"] = float((t[:, :, 0].max(1) - t[:, :, 0].min(1)).mean())
    res["wave_end_skew_mean"] = float((t[:, :, 12].max(1) - t[:, :, 12].min(1)).mean())
    hw = t[:, 0, 15]
    cu_key = (t[:, 0, 14] & 0xF) * 256 + ((hw >> 8) & 0xFF)    # XCC, then CU / SH / SE bits of HW_ID
    span = int(t[:, :, 12].max() - t[:, :, 0].min())
    res["kernel_span_cycles"] = span
    gaps, per_cu = [], {}
    for b in range(blocks):
        per_cu.setdefault(int(cu_key[b]), []).append((int(t[b, :, 0].min()), int(t[b, :, 12].max())))
    for v in per_cu.values():
        v.sort()
        gaps += [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
    res["distinct_hw_ids"] = len(per_cu)
    res["blocks_per_hw_id_max"] = max(len(v) for v in per_cu.values())
    if gaps:
        g = np.array(gaps)
        res["gap_between_blocks_median"] = float(np.median(g))
        res["gap_negative_frac"] = float((g < 0).mean())
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
