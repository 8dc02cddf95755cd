#!/usr/bin/env python3
"""Cold-cache determinism check of k_final forms.

The removed round-4 prefetch form of k_final differed on the FIRST render of
a process -- one 16-lane group at one sample -- and matched on the later ones.
A first render runs with cold L2 / Infinity-Cache lines and longer gather
latencies.  This tool makes every render cold: before each one it streams a
buffer larger than the 256 MB Infinity Cache through the device (fill + sum),
so the embedding rows a render gathers come from HBM again.  Each render's
outputs (image, depth, weights_sum, samvit, head-input rows) are compared with
a warm reference render of the same library and form; the differing rays and
the 16-lane groups they fall into are printed.

usage (GPU box): [SAMNERF_LIB=lib.so] python tools/cold_render_check.py --reps 12 [--env K=V ...]
  --ref-env K=V  environment of the reference render (default: the same as --env)
  --no-cold      skip the cache flush (warm renders)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "segment-anything-nerf_amd"), os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--ref-env", action="append", default=None)
    ap.add_argument("--no-cold", action="store_true")
    ap.add_argument("--head-mode", type=int, default=0)
    ap.add_argument("--view-width", type=int, default=0)
    ap.add_argument("--taps", action="store_true",
                    help="render with the parity taps: report the differing samples (sigma2) and "
                         "whether k_final's corner rows (rows2, every ray) differ too")
    a = ap.parse_args()
    from helpers import make_net
    from oracle import synth
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, ROW
    dev = torch.device("cuda", 0)

    def setenv(pairs):
        for kv in pairs:
            k, v = kv.split("=", 1)
            os.environ[k] = v

    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=23, emb_scale=0.5, ln_jitter=0.1), dev)
    pose, intr = synth.gui_camera(512, 80, rot=synth.random_rotation(11))
    ro, rd = ops.get_rays(pose, intr, 80, 512, device=dev)
    flush = torch.empty(512 * 1024 * 1024, dtype=torch.float32, device=dev)   # 2 GiB

    def render():
        fr = FusedRenderer(net, head_mode=a.head_mode)
        rows = torch.empty(ro.shape[0], ROW, device=dev)
        o = fr.render(ro, rd, rows=rows, view_width=a.view_width, taps=bool(a.taps))
        o.pop("tap_rays", None)
        o["rows"] = rows
        torch.cuda.synchronize()
        return {k: v.detach().cpu().clone() for k, v in o.items()}

    first = None
    setenv(a.env)
    outs = []
    for i in range(a.reps):
        if not a.no_cold:
            flush.fill_(float(i))
            torch.cuda.synchronize()
        outs.append(render())
        if first is None:
            first = outs[0]
    setenv(a.ref_env if a.ref_env is not None else a.env)
    ref = render()                       # warm: right after the others
    bad = 0
    for i, o in enumerate(outs):
        diffs = {}
        rays = set()
        for k in ref:
            ne = o[k] != ref[k]
            if ne.dim() > 1:
                ne = ne.reshape(ne.shape[0], -1).any(1)
            if ne.any():
                diffs[k] = int(ne.sum())
                rays.update(ne.nonzero().flatten().tolist())
        if diffs:
            bad += 1
            rs = sorted(rays)
            groups = sorted({r // 16 for r in rs})
            print(f"render {i}: DIFFERS {diffs}; rays {rs[:8]}{'...' if len(rs) > 8 else ''} "
                  f"in {len(groups)} 16-ray groups {groups[:6]}", flush=True)
            if a.taps and "sigma2" in diffs:
                ne = (o["sigma2"] != ref["sigma2"]).nonzero()[:6].tolist()
                rel = ((o["sigma2"] - ref["sigma2"]).abs() / ref["sigma2"].abs().clamp_min(1e-30)).max().item()
                print(f"    sigma2 (ray, sample) {ne}, max rel {rel:.3g}; corner rows equal: "
                      f"{'rows2' not in diffs}; positions equal: {'u2' not in diffs}", flush=True)
        else:
            print(f"render {i}: equal", flush=True)
    print(f"SUMMARY env={a.env} cold={not a.no_cold} reps={a.reps} differing_renders={bad}")


if __name__ == "__main__":
    main()
