#!/usr/bin/env python3
"""Headline view time and shader clock against burst length: bursts of K
views back to back (K = 8 .. 200, 1 and 2 views in flight), each bracketed by
samnerf_clock_stamp launches (bench.timed_clock), an idle second between
bursts.  Question it answers: is the gap between bench.py's tuning rounds (8
views) and its timed region (20 views) the power controller lowering the
clock over a longer burst.  usage (GPU box): python tools/burst_clock.py"""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "segment-anything-nerf_amd"))


def main():
    import bench
    from samnerf_amd import ops, synth
    from samnerf_amd._lib import lib
    from samnerf_amd.fused import FusedRenderer
    dev = torch.device("cuda", 0)
    net, _, _ = bench.build_net(True, dev)
    pose, intr = synth.gui_camera(512, 512)
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    frs = [FusedRenderer(net), FusedRenderer(net)]

    def view(i, n):
        with torch.cuda.stream(streams[i % n]):
            return frs[i % n].render(ro, rd, view_width=512)

    for i in range(10):
        view(i, 2)
    torch.cuda.synchronize()
    stamps = torch.zeros(2, 768, dtype=torch.int64, device=dev)
    cur = streams[0]
    rows = []
    for rnd in range(2):
        for n in (1, 2):
            for k in (8, 20, 60, 200):
                time.sleep(1.0)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                lib().samnerf_clock_stamp(ctypes.c_void_p(stamps[0].data_ptr()), ctypes.c_void_p(cur.cuda_stream))
                for i in range(k):
                    view(i, n)
                cur.wait_stream(streams[1])
                lib().samnerf_clock_stamp(ctypes.c_void_p(stamps[1].data_ptr()), ctypes.c_void_p(cur.cuda_stream))
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                clk = bench.timed_clock(stamps.cpu().numpy())
                r = {"round": rnd, "streams": n, "views": k, "ms_per_view": dt * 1e3 / k,
                     "clock_ghz": clk.get("ghz") if isinstance(clk, dict) else clk}
                rows.append(r)
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
