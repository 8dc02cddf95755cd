#!/usr/bin/env python3
"""Benchmark: rays/s of the fused ray-march hot path at 512x512 (+ SAM feature).

Workload (BASELINE.json configs[2] = "garden --with_sam: RGB + 256-dim SAM
feature head, 512x512, 1xMI355X"): one STEP renders one 512x512 GUI view
(262,144 rays: get_rays + 3 proposal rounds 128/64/32 + hash grids + MLPs +
compositing + 256-d SAM head per ray) on synthetic random-init weights of the
reference architecture.  With --gpus N > 1 the view's rows are split into N
equal bands, one rank per GPU (strong scaling on a fixed view), and the packed
per-ray outputs [rays/N, 3+1+1+256] are all-gathered over RCCL, as BASELINE
config 4 / SURVEY.md 8e describe.  `python bench.py --gpus N` starts the N
ranks itself (torch.distributed.run, as a child process) when it is not
already running under a launcher.  Each step is one full view on every rank;
view i's all-gather runs behind view i+1's kernels, and the last view's
gather completes inside the timed region.  The headline gathers fp32 (exact);
the lossy q16 transport is timed after it and reported beside it.

Prints ONE JSON line (rank 0).  `value` = rays of the whole view x steps /
(max over ranks of the timed region).  `roofline` prices the dominant kernel
against the guide peak of the unit closest to saturation (L2 bandwidth on the
algorithmic bytes, VALU issue or MFMA issue) from HIP events
recorded on the launch stream, with the per-ray counter rates of the
committed PMC passes (profiles/pmc_rates.json); `cpu_baseline` times the CPU
oracle (torch-CPU restatement of the reference renderer + C restatement of its encoders) on the view's rays, and
`parity_vs_ref` compares a parity-weight render of the same view with it.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "segment-anything-nerf_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "rays/sec (RGB+256-d SAM feat) at 512×512, 1/2/4/8 MI355X; PSNR vs ref"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
L2_PEAK_GBS = 34500.0          # MI355X_MICROARCH.md: L2 ~34.5 TB/s aggregate
CLOCK_GHZ = 2.4                # MI355X_MICROARCH.md: max clock
N_CU, N_SIMD = 256, 1024
# Per-stage counter rates of one view (tools/pmc_rates.py over the rocprofv3
# PMC passes of tools/pmc_passes.sh; recomputable from the PMC table committed
# beside it): VALU-issue and MFMA-busy cycles per ray, HBM bytes per ray.
PMC_RATES = os.path.join(REPO, "profiles", "pmc_rates.json")
# The texture-address rate is not one number: tools/ta_rate.hip measured
# 0.45 lane-addresses/clk/CU for random dword gathers (one 128-B line per lane)
# and 14.6 for contiguous ones (profiles/r3_ta_rate.json), so the gather
# stages are priced against the guide's L2 bandwidth and their VALU issue
# rate instead, and `bound` names whichever is closer to its peak.

# Algorithmic bytes per ray and stage (SURVEY.md 8d / BASELINE.md 3): fp32
# embedding gathers (8 corners x C x 4 B per level per sample) + the stage's
# own ray I/O.  Intermediates that stay in L2 are not counted.
STAGES = ["prop0", "prop1", "final", "s_grid", "sam_head"]
ALG_BYTES_PER_RAY = {
    "prop0": 128 * 5 * 8 * 2 * 4 + 24 + 65 * 4,            # gathers + rays in + bins out
    "prop1": 64 * 5 * 8 * 2 * 4 + 65 * 4 + 33 * 4,
    "final": 32 * 16 * 8 * 2 * 4 + 24 + 33 * 4 + 20 + 31 * 4,
    "s_grid": 32 * 16 * 8 * 8 * 4 + 32 * 4 * 4 + 128 * 4,
    "sam_head": 164 * 4 + 256 * 4,
}
ALG_BYTES_RAY_TOTAL = 226_348
# SAM head (network.py:36-75): 163->256, 256->256, 419->256, 256->256, 256->256
HEAD_FLOP_PER_RAY = 2 * 256 * (163 + 256 + 419 + 256 + 256)  # 691,200
# MFMA issue cycles of the SAM head's structure per 32 rays: f16x3 on the
# product's k_sam_head_w8 (two 16-ray waves: 44 32-deep k-blocks -- K padded
# 192 + 256 + 448 + 256 + 256 -- x 16 output tiles x 3 fp16 products on
# v_mfma_f32_16x16x32_f16, 16 cycles; round 5's k_sam_head_h16q: 86 16-deep
# k-blocks x 8 tiles x 3 x 32 cycles); exact mode: 688 k-steps of 2 x 8 tiles
# on v_mfma_f32_32x32x2_f32 (64 cycles)
HEAD_MFMA_CYCLES_PER_32 = {0: 2 * 44 * 16 * 3 * 16, 1: 688 * 8 * 64}
BF16_MFMA_PEAK_TFS = 2500.0    # MI355X_MICROARCH.md: dense BF16/F16 ~2.5 PF
F32_MFMA_PEAK_TFS = 157.3      # MI355X_MICROARCH.md: F32 matrix = vector peak
DTYPE = {0: "fp32-equivalent: fp32 in the reference's op order for everything that decides a "
            "discrete result (near/far, bins, proposal grids + MLPs, compositing, sample_pdf); "
            "grid_mlp (32->64->64->16 per sample), the SAM head (163->256x5) and the mask head "
            "(143->256->256->K per sample) as f16x3: each fp32 product as three fp16 MFMA products on "
            "power-of-two scaled operands, fp32 accumulate -- error vs float64 at the level of exact "
            "fp32 GEMMs (csrc/f16x3.h, tests/test_gpu_render.py); view_mlp on fp32 MFMA",
         1: "fp32 throughout: grid_mlp, view_mlp, the SAM head and the mask head on fp32 MFMA "
            "(v_mfma_f32_32x32x2_f32), the rest in the reference's op order"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without a launcher environment bench.py starts them")
    ap.add_argument("--steps", type=int, default=30)           # 30 views: ~0.1 s timed, steadier than 10
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--W", type=int, default=512)
    ap.add_argument("--no-sam", action="store_true", help="config 2 (RGB only)")
    ap.add_argument("--cpu-rays", type=int, default=262144,
                    help="rays in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--ref-gpu-rays", type=int, default=262144,
                    help="rays of the view rendered by run_torch, the reference's unfused op "
                         "sequence on the same GPU (0 = skip)")
    ap.add_argument("--head-mode", type=int, default=0,
                    help="0 = f16x3 (fp32-equivalent) grid_mlp + SAM / mask heads (default), "
                         "1 = exact fp32 MFMA")
    ap.add_argument("--no-alt", action="store_true",
                    help="skip the side measurements after the headline (exact-fp32 precision at "
                         "N=1, q16 transport at N>1)")
    ap.add_argument("--chunks", type=int, default=0,
                    help="N > 1: 0 = one launch per view with its all-gather pipelined behind "
                         "the next view's rendering; k > 0 = k row chunks per view, each "
                         "chunk's all-gather behind the next chunk")
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams the views are issued on round-robin, so view i+1's kernels "
                         "overlap view i's (each stream has its own workspace).  0 = tuned in the "
                         "warm-up between the two counts around 1 (whole view) / 2 (2 ranks) / 3 "
                         "(4-8 ranks) (measured, DESIGN.md 7)")
    ap.add_argument("--mode", choices=["render", "train", "gui", "rgbtrain"], default="render",
                    help="render: cfg 3 view throughput (the headline metric); train: cfg 5 "
                         "SAM-feature distillation step (4096 rays, forward + backward + Adam); "
                         "gui: the reference GUI's frame (readme.md:5) -- 512x512 RGB + 64x64 "
                         "SAM-feature render")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL); gloo for rehearsals")
    ap.add_argument("--share-gpu", action="store_true",
                    help="all ranks on GPU 0 (rehearsal of the N-rank path on a one-GPU box)")
    ap.add_argument("--rank-share", type=int, default=0,
                    help="one GPU renders only the row band rank --share-rank of N = this value "
                         "would render in an N-rank strong-scaled view (the 512x512 camera, not a "
                         "smaller view): the per-rank load of the N-GPU bench; value = that band's "
                         "rays/s")
    ap.add_argument("--share-rank", type=int, default=-1, help="band index for --rank-share (default N//2)")
    ap.add_argument("--gather-codec", choices=["fp32", "q16"], default="fp32",
                    help="transport of the headline's per-view all-gather at N > 1 "
                         "(samnerf_amd/dist.py): fp32 = 1,044 B/ray, exact (default); q16 = 536 B/ray "
                         "records, samvit as int16 with a per-ray power-of-two scale (|err| <= 2^-14 "
                         "of the ray's max, own band exact).  The other codec is timed after the "
                         "headline and reported beside it (unless --no-alt)")
    ap.add_argument("--train-head", choices=["hip", "torch"], default="hip",
                    help="--mode train: the SAM head's forward + backward on the HIP kernels "
                         "(sam_head_train.hip) or as torch ops with autograd (comparison)")
    ap.add_argument("--torch-adam", action="store_true",
                    help="--mode train: torch.optim.Adam (foreach) instead of the one-pass HIP Adam")
    ap.add_argument("--scene", choices=["default", "surface"], default="default",
                    help="weights of the timed view: default-init (the headline, embeddings U(+-1e-4) as "
                         "the reference initialises them) or the opaque-sphere scene "
                         "(synth.make_surface_params: rays saturate at a surface, as in a trained scene)")
    ap.add_argument("--no-tiles", dest="tiles", action="store_false",
                    help="row-major ray waves instead of 8x4 pixel tiles (samnerf_model.view_width = 0)")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def maybe_launch(args):
    """`--gpus N` > 1 outside a torch.distributed launcher: start the N ranks
    (torch.distributed.run on 127.0.0.1, one process per GPU) as a child
    process and return its exit status.  Runs before anything touches the
    GPU; returns None when this process is already a rank (or N = 1)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC for RCCL on this host
    return subprocess.call(cmd, env=env)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; run "
                         f"`python bench.py --gpus {args.gpus}` (it launches the ranks) or a "
                         f"launcher with --nproc-per-node {args.gpus}")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # --dist-backend gloo --share-gpu: a rehearsal of the multi-rank code
        # path with every rank on GPU 0 (RCCL needs one GPU per rank)
        dev_index = 0 if args.share_gpu else local
        torch.cuda.set_device(dev_index)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(args.dist_backend, rank=rank, world_size=world)
        return rank, world, torch.device("cuda", dev_index)
    torch.cuda.set_device(0)
    return rank, world, torch.device("cuda", 0)


def build_net(with_sam, device, seed=0, emb_scale=1e-4, surface=False):
    """NeRFNetwork with synthesised weights: the bench's default-init scene
    (embeddings U(+-1e-4) as grid.py:144-146), with emb_scale 0.5 the
    parity-weight scene of the tests, with surface=True the
    opaque-sphere scene of the N1 line (synth.make_surface_params)."""
    from nerf.network import NeRFNetwork, default_opt
    from samnerf_amd import synth
    spec = synth.ModelSpec(with_sam=with_sam)
    if surface:
        params = synth.make_surface_params(spec, seed=seed)
    else:
        params = synth.make_params(spec, seed=seed, emb_scale=emb_scale, ln_jitter=0.0)
    net = NeRFNetwork(default_opt(with_sam=with_sam))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    return net.to(device).eval(), spec, params


def cpu_baseline(spec, params, pose, intr, H, W, n_rays, gpu_out=None):
    """Time the CPU oracle on n_rays rays spread over the same view; with the
    GPU outputs of that view, also return PSNR / max error of the GPU render
    against it (the metric's "PSNR vs ref"; psnr formula of utils.py:347-357)."""
    from oracle import renderer as orc
    # the box exposes every host CPU but grants this job a share of them
    # (OMP_NUM_THREADS, 16 per GPU); use the share, not the machine
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    torch.set_num_threads(threads)
    ro, rd = orc.get_rays(pose, intr, H, W)
    idx = torch.linspace(0, H * W - 1, n_rays).long()          # rays spread over the view
    model = orc.OracleNeRF(spec, params)
    model.run(ro[idx[:64]], rd[idx[:64]], return_feats=1)      # warm-up
    t0 = time.perf_counter()
    ref = model.render(ro[idx], rd[idx], return_feats=1)
    dt = time.perf_counter() - t0
    res = {"value": n_rays / dt, "unit": "rays/s", "cores": threads, "kind": "port",
           "sample": f"{n_rays} rays of the {H}x{W} view (same weights, chunks of 16384 as renderer.py:195); torch-CPU "
                     f"restatement of nerf/renderer.py+network.py, encoders in C "
                     f"(OpenMP over points); {dt:.1f} s"}
    parity = None
    if gpu_out is not None:
        g = {k: v.detach().float().cpu() for k, v in gpu_out.items()}
        img_g, img_r = g["image"][idx], ref["image"].reshape(-1, 3)
        mse = float(((img_g - img_r) ** 2).mean())
        parity = {"rays": n_rays, "weights": "parity weights: embeddings U(+-0.5), seed 33 (tests/, SURVEY.md 8c)",
                  "psnr_image_db": float("inf") if mse == 0 else -10.0 * float(np.log10(mse)),
                  "max_abs_image": float((img_g - img_r).abs().max()),
                  "max_abs_depth_rel": float(((g["depth"][idx] - ref["depth"].reshape(-1)).abs()
                                              / ref["depth"].reshape(-1).abs().clamp_min(1.0)).max())}
        if "samvit" in g and "samvit" in ref:
            parity["max_abs_samvit"] = float((g["samvit"][idx] - ref["samvit"].reshape(n_rays, -1)).abs().max())
    return res, parity


def reference_equivalent_gpu(net, ro, rd, n_rays, chunk=16384):
    """The reference's own op sequence on the same GPU: NeRFRenderer.run_torch
    (renderer.py:221-390 as ~350 torch ops per chunk, hash/SH encoders = the
    drop-in HIP kernels with the reference's one-thread-per-(point, level)
    design), staged in max_ray_batch = 16384 chunks like renderer.py:195.
    This is BASELINE.md's "reference-equivalent single-GPU" denominator of the
    >= 10x target (the reference's CUDA extensions cannot run here)."""
    n = min(n_rays, ro.shape[0])
    with torch.no_grad():
        net.run_torch(ro[:chunk], rd[:chunk], return_feats=1)          # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for h in range(0, n, chunk):
            net.run_torch(ro[h:h + chunk], rd[h:h + chunk], return_feats=1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "rays/s", "rays": n,
            "what": "NeRFRenderer.run_torch (the reference's unfused torch op sequence, drop-in HIP "
                    "encoders), chunks of 16384 rays, same view and weights"}


def mask_view(dev, steps, warmup, head_mode=0, ref_rays=32768):
    """--with_mask rendering (mask_mlp_type 'default', n_inst 2, RGB + instance
    logits, no SAM; renderer.py:392-395, :451-452) of one 512 x 512 view:
    the fused render + k_mask_head against the reference's unfused op
    sequence (run_torch, return_mask=1) on the same GPU (`ref_rays` of the
    view, chunks of 16384).  Returns the side-line dict."""
    from nerf.network import NeRFNetwork, default_opt
    from samnerf_amd import ops, synth
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="default", sum_after_mlp=False)
    params = synth.make_params(spec, seed=0, emb_scale=1e-4)
    net = NeRFNetwork(default_opt(with_sam=False, with_mask=True, mask_mlp_type="default", n_inst=2))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    net = net.to(dev).eval()
    H = W = 512
    pose, intr = synth.gui_camera(W, H)
    fr = FusedRenderer(net, head_mode=head_mode)

    def view():
        ro, rd = ops.get_rays(pose, intr, H, W, device=dev)
        return fr.render(ro, rd, mask=True, view_width=W)

    for _ in range(warmup):
        view()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = view()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    # the same view without the instance logits: the difference is the mask
    # head's share (k_mask_head + the per-sample geo_feat stores)
    for _ in range(warmup):
        fr.render(*ops.get_rays(pose, intr, H, W, device=dev), mask=False, view_width=W)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fr.render(*ops.get_rays(pose, intr, H, W, device=dev), mask=False, view_width=W)
    torch.cuda.synchronize()
    dt_nomask = (time.perf_counter() - t0) / steps
    head_ms = (dt - dt_nomask) * 1e3
    # f16x3: 3 fp16 MFMA products per fp32 product of 143->256->256->32 (the
    # padded output tile) per sample, 32 samples per ray
    head_flop = 3 * 2 * (144 * 256 + 256 * 256 + 256 * 32) * 32 * H * W
    ro, rd = ops.get_rays(pose, intr, H, W, device=dev)
    n, chunk = min(ref_rays, H * W), 16384
    with torch.no_grad():
        ref = net.run_torch(ro[:chunk], rd[:chunk], return_mask=1)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for h in range(0, n, chunk):
            ref = net.run_torch(ro[h:h + chunk], rd[h:h + chunk], return_mask=1)
        torch.cuda.synchronize()
        dt_ref = (time.perf_counter() - t1) / n
    err = (out["instance_mask_logits"][n - chunk:n] - ref["instance_mask_logits"]).abs().max().item()
    return {"value": H * W / dt, "unit": "rays/s", "ms_per_step": dt * 1e3,
            "reference_equivalent_gpu": {"value": 1.0 / dt_ref, "unit": "rays/s", "rays": n},
            "speedup": (H * W / dt) * dt_ref,
            "max_abs_logits_vs_unfused": err, "dtype": DTYPE[head_mode],
            "ms_without_mask": dt_nomask * 1e3, "mask_head_ms": head_ms,
            # fingerprint of the full view's logits (bit-identity of A/B builds)
            "logits_sha16": hashlib.sha256(out["instance_mask_logits"].cpu().numpy().tobytes()).hexdigest()[:16],
            "mask_head_mfma_frac": (head_flop / (head_ms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFS
                                    if head_mode == 0 and head_ms > 0 else None),
            "what": "--with_mask 'default' head (m_grid L16C8 + SkipConnMLP 143->256->256->2 per sample, "
                    "weighted sum): fused render + k_mask_head vs run_torch(return_mask=1), 512x512 view"}


def train_steps(dev, steps, warmup, torch_adam=False, head="hip", deterministic=False):
    """BASELINE config 5: one step = fused forward of 4096 rays
    (64x64, fovy 60) with grad, MSE vs a N(0,1) [1,256,64,64] target (seed 1)
    after the reference's bilinear resize, backward (HIP s_grid scatter +
    torch head), Adam(lr 1e-2, eps 1e-15) with the RGB parameters frozen
    (main.py:255-262, 296; utils.py:1072-1106).  Returns (ms per step, loss)."""
    import torch.nn.functional as F
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, render_sam_train
    from samnerf_amd.optim import FusedAdam
    from samnerf_amd import synth
    net, spec, params = build_net(True, dev)
    net.train()
    for k, p in net.named_parameters():
        p.requires_grad = k.startswith("s_grid") or k.startswith("samvit_mlp")
    params_ = [p for p in net.parameters() if p.requires_grad]
    opt = (torch.optim.Adam(params_, lr=1e-2, eps=1e-15) if torch_adam
           else FusedAdam(params_, lr=1e-2, eps=1e-15))
    renderer = FusedRenderer(net, deterministic=deterministic)
    h = w = 64
    pose, intr = synth.gui_camera(w, h)
    ro, rd = ops.get_rays(pose, intr, h, w, device=dev)
    g = torch.Generator(device="cpu").manual_seed(1)
    gt = torch.randn(1, 256, 64, 64, generator=g).to(dev)

    def step():
        out = render_sam_train(renderer, ro, rd, view_width=w, head=head)
        pred = out["samvit"].reshape(1, h, w, 256).permute(0, 3, 1, 2).contiguous()
        pred = F.interpolate(pred, gt.shape[2:], mode="bilinear")
        loss = F.mse_loss(pred, gt)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return dt * 1e3 / steps, float(loss.detach())


def rgb_train_steps(dev, steps, warmup, fused=True, h=64, w=128):
    """One RGB training step (utils.py:897-937, the reference's first training
    stage): 8,192 rays -- the batch adaptive_num_rays settles on for
    num_points = 2^18 (main.py:96, 226) -- of a parity-weight scene at the
    reference's table sizes, perturbed sampling, MSE + proposal + distortion
    losses, backward, Adam(lr 1e-2, eps 1e-15) over every group of get_params
    (main.py:296).  fused: samnerf_rgb_train_step (rgb_train.hip); else the
    torch path (run_torch + autograd with the drop-in encoder kernels).
    Returns (ms per step, final loss)."""
    from samnerf_amd import ops, synth
    from samnerf_amd.optim import FusedAdam
    from samnerf_amd.train import rgb_train_step, rgb_train_step_fused
    net, _, _ = build_net(False, dev, seed=3, emb_scale=0.5)
    net.train()
    net.fused = fused          # False: NeRFRenderer.run_torch under autograd
    net.opt.adaptive_num_rays = False
    opt = FusedAdam(net.get_params(1e-2), eps=1e-15)
    # the reference's training batch: N rays at random pixels of a view
    # (utils.py:get_rays with N > 0, torch.randint over H * W), here of a 512^2
    # GUI view -- not neighbours in the image, so the scatter merges along rays
    pose, intr = synth.gui_camera(512, 512)
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)
    inds = torch.randint(0, 512 * 512, (h * w,), generator=torch.Generator().manual_seed(4)).to(dev)
    ro, rd = ro[inds].contiguous(), rd[inds].contiguous()
    gt = torch.rand(ro.shape[0], 3, generator=torch.Generator().manual_seed(4)).to(dev)

    def step(i):
        if fused:
            _, loss, _ = rgb_train_step_fused(net, ro, rd, gt, global_step=1 + i)
        else:
            _, loss, _ = rgb_train_step(net, ro, rd, gt, global_step=1 + i)
            for p in net.parameters():
                p.grad = None
            loss.backward()
        opt.step()
        return loss

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(warmup + i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps, float(loss.detach())


def mask_train_steps(dev, steps, warmup, fused=True, n_rays=4096):
    """One --with_mask training step (utils.py:941-977; main.py:255-262: only
    m_grid and mask_mlp train): 4,096 rays at random pixels of a 512^2 view of
    a 'default'-head mask model (n_inst 2) at the reference's table sizes,
    render with return_mask=1, softmax / clamp / NLL of random labels,
    backward, Adam(lr 1e-2, eps 1e-15).  fused: the HIP mask-training kernels
    (mask_head_train.hip); else the torch path (run_torch + autograd with the
    drop-in encoder kernels).  Returns (ms per step, final loss)."""
    from nerf.network import NeRFNetwork, default_opt
    from samnerf_amd import ops, synth
    from samnerf_amd.optim import FusedAdam
    from samnerf_amd.train import mask_train_step
    spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="default", sum_after_mlp=False)
    params = synth.make_params(spec, seed=5, emb_scale=0.5)
    net = NeRFNetwork(default_opt(with_sam=False, with_mask=True, mask_mlp_type="default", n_inst=2))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    net = net.to(dev).train()
    net.fused = fused
    for k, p in net.named_parameters():
        p.requires_grad = k.startswith("m_grid") or k.startswith("mask_mlp")
    opt = FusedAdam([p for p in net.parameters() if p.requires_grad], lr=1e-2, eps=1e-15)
    pose, intr = synth.gui_camera(512, 512)
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=dev)
    inds = torch.randint(0, 512 * 512, (n_rays,), generator=torch.Generator().manual_seed(6)).to(dev)
    ro, rd = ro[inds].contiguous(), rd[inds].contiguous()
    gt = torch.randint(0, 2, (n_rays,), generator=torch.Generator().manual_seed(7)).to(dev)

    def step():
        _, loss = mask_train_step(net, ro, rd, gt)
        for p in net.parameters():
            p.grad = None
        loss.backward()
        opt.step()
        return loss

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps, float(loss.detach())


RGB_TRAIN_WHAT = {
    "dtype": "fp32 throughout (forward in the fused render's op order, grid_mlp / view_mlp exact fp32; "
             "hand-written backward; grid gradients by fp32 atomics)",
    "data": "synthetic parity-weight scene (embeddings U(+-0.5)) at the reference's table sizes, "
            "U(0,1) target colours",
    "config": {"workload": "RGB training step (utils.py:897-937): 8192 rays at random pixels of a 512x512 "
                           "view, perturb, MSE + proposal + distortion losses, backward, Adam over all groups",
               "optimizer": "FusedAdam lr 1e-2 eps 1e-15"},
}


def rgb_train_main(args, dev):
    ms, loss = rgb_train_steps(dev, args.steps, args.warmup, fused=True)
    ms_t, _ = rgb_train_steps(dev, max(3, args.steps // 2), 2, fused=False)
    rec = {"metric": "RGB training steps/s (8192 rays, fwd+bwd+Adam)", "value": 1e3 / ms,
           "unit": "steps/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": ms, "higher_is_better": True, "rays_per_s": 8192 * 1e3 / ms,
           "final_loss": loss, "torch_path_ms_per_step": ms_t, "speedup_vs_torch_path": ms_t / ms,
           **RGB_TRAIN_WHAT, "vs_baseline": None}
    print(json.dumps(rec), flush=True)


TRAIN_WHAT = {
    "optimizer": "FusedAdam: one-pass HIP Adam (train_optim.hip), torch.optim.Adam semantics",
    "dtype": "fp32 (fused render forward: grid_mlp f16x3 MFMA (fp32-equivalent); SAM head forward + backward on exact "
             "fp32 MFMA, sam_head_train.hip; s_grid scatter fp32 atomics)",
    "data": "synthetic (default-init weights, N(0,1) target)",
    "config": {"workload": "cfg5: 64x64 rays, with_sam, RGB frozen", "optimizer": "Adam lr 1e-2 eps 1e-15"},
}


def train_main(args, dev):
    ms, loss = train_steps(dev, args.steps, args.warmup, args.torch_adam, args.train_head)
    rec = {"metric": "cfg5 SAM distillation train steps/s (4096 rays, fwd+bwd+Adam)",
           "value": 1e3 / ms, "unit": "steps/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
           "rays_per_s": 4096 * 1e3 / ms, "final_loss": loss, **TRAIN_WHAT, "vs_baseline": None}
    if args.torch_adam:
        rec["optimizer"] = "torch.optim.Adam (foreach)"
    if args.train_head == "torch":
        rec["dtype"] = "fp32 (fused render forward: grid_mlp f16x3 MFMA; SAM head torch autograd)"
    print(json.dumps(rec), flush=True)


def gui_frame_time(dev, H, W, steps, warmup, net=None):
    """Seconds per GUI frame (nerf/gui.py:143-161 -> utils.py:1647-1712): the
    H x W view without features plus the 64 x 64 feature rays."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    from samnerf_amd import synth
    if net is None:
        net, _, _ = build_net(True, dev)
    r = FusedRenderer(net)
    pose, intr = synth.gui_camera(W, H)
    pose_lr, intr_lr = synth.gui_camera(64, 64)

    def frame():
        ro, rd = ops.get_rays(pose, intr, H, W, device=dev)
        img = r.render(ro, rd, feats=False, view_width=W)
        ro2, rd2 = ops.get_rays(pose_lr, intr_lr, 64, 64, device=dev)
        return img, r.render(ro2, rd2, view_width=64)

    for _ in range(warmup):
        frame()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        frame()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def gui_main(args, dev):
    """The reference GUI's per-frame render work (nerf/gui.py:143-161 ->
    utils.py:1647-1712 test_gui -> test_step): the H x W view without
    features (return_feats=0: the reference still computes and drops them,
    the fused path skips them) plus the 64 x 64 feature rays for the SAM
    decoder.  readme.md:5 quotes 5 FPS on a V100 for this loop including the
    decoder (not run here)."""
    H, W = args.H, args.W
    dt = gui_frame_time(dev, H, W, args.steps, args.warmup)
    rays = H * W + 64 * 64
    print(json.dumps({
        "metric": "GUI frame: 512x512 RGB + 64x64 SAM-feature render (frames/s)", "value": 1.0 / dt,
        "unit": "frames/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt * 1e3, "higher_is_better": True, "rays_per_s": rays / dt,
        "dtype": "fp32-equivalent (SAM head: f16x3 MFMA, fp32 accumulate)",
        "data": "synthetic (random-init weights of the reference architecture, GUI camera)",
        "config": {"workload": f"{H}x{W} RGB (features skipped) + 64x64 with 256-d SAM features",
                   "reference": "readme.md:5: 5 FPS on V100 incl. the SAM decoder"},
        "vs_baseline": None}), flush=True)


class ViewRunner:
    """Issues views of this rank's row band on `n_streams` HIP streams (each
    with its own workspace) and, at N > 1, all-gathers each view through a
    ShardedViewPipeline (view i's gather behind view i+1's kernels)."""

    def __init__(self, args, renderer, world, dev, H, W, pose, intr, r0, r1, codec):
        from samnerf_amd.dist import ShardedViewPipeline
        self.args, self.renderer, self.world, self.dev = args, renderer, world, dev
        self.H, self.W, self.pose, self.intr, self.r0, self.r1 = H, W, pose, intr, r0, r1
        self.chunks = max(1, args.chunks) if world > 1 else 1
        # Views in flight (tools/streams_ab.sh): on the
        # default scene the whole view is fastest on 1 stream (2.785 vs 2.81 ms
        # on 2: the chip is at its power limit, so a second view in flight only
        # shares it), a half view on 2, a quarter or an eighth on 3; on the
        # opaque-sphere scene (L2-miss latency) the whole view gains 13 % from a
        # second stream.  --streams 0 (default): the warm-up times the two
        # candidate counts around that rule on the workload itself and the timed
        # views use the faster (max over ranks, so every rank picks the same);
        # --rank-share N picks as N ranks would.
        eff = args.rank_share if world == 1 and args.rank_share > 1 else world
        rule = 1 if eff == 1 else 2 if eff == 2 else 3
        self.cands = ([1, 2] if rule == 1 else [2, 3]) if not args.streams else [args.streams]
        self.n_active = args.streams or rule
        self.tuned = None
        self.tuned_clock = None
        self.clock = None
        self.streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev)
                                                           for _ in range(max(self.cands) - 1)]
        self.n_step = 0
        # fp32 transport: each rank renders its band straight into its slice of
        # the gather buffer (samnerf_render_forward_tile), no pack copy
        keys = ("image", "depth", "weights_sum") + (() if args.no_sam else ("samvit",))
        tile_cols = (5 if args.no_sam else 261) if codec == "fp32" else None
        self.pipe = (ShardedViewPipeline(renderer.render, H, W, keys=keys, codec=codec, tile_cols=tile_cols)
                     if world > 1 and args.chunks == 0 else None)

    def _step_on_stream(self, raws=None):
        from samnerf_amd import ops
        from samnerf_amd._lib import lib
        from samnerf_amd.dist import render_view_sharded
        it = iter(raws or [])
        H, W, dev = self.H, self.W, self.dev

        def ray_fn(row0, rows):
            return ops.get_rays(self.pose, self.intr, H, W, device=dev, row0=row0, rows=rows)

        def render_fn(ro, rd, out_tile=None):
            raw = next(it, None)
            lib().samnerf_set_stage_events(raw, 6 if raw is not None else 0)
            return self.renderer.render(ro, rd, view_width=W if self.args.tiles else 0, out_tile=out_tile)

        if self.world > 1 and self.args.chunks > 0:
            return render_view_sharded(render_fn, ray_fn, H, W, chunks=self.chunks)
        if self.world > 1:
            self.pipe.submit(ray_fn, render_fn)   # this view's gather overlaps the next view
            return self.pipe.collect_ready()
        return render_fn(*ray_fn(self.r0, self.r1 - self.r0))

    def step(self, raws=None):
        s = self.streams[self.n_step % self.n_active]
        self.n_step += 1
        with torch.cuda.stream(s):
            return self._step_on_stream(raws)

    def _flush(self):
        return self.pipe.flush() if self.pipe is not None else []

    def run(self, steps, warmup, stages=True):
        """Warm up, then time exactly `steps` views bracketed by a barrier and
        a device synchronisation on both sides; returns (max-over-ranks
        seconds, the last view's outputs, per-stage ms, their source)."""
        from samnerf_amd._lib import lib
        import ctypes

        def make_event_set():
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
            for e in evs:                      # create the underlying hipEvent_t
                e.record()
            raw = (ctypes.c_void_p * 6)(*[e.cuda_event for e in evs])
            return evs, raw

        # the warm-up runs on every candidate stream (each allocates its
        # workspace on first use, outside the tuning and the timed views)
        n_keep, self.n_active = self.n_active, max(self.cands)
        for _ in range(max(warmup, self.n_active)):
            self.step()
        self._flush()
        self.n_active, self.n_step = n_keep, 0
        if len(self.cands) > 1:
            # views in flight: time each candidate stream count on this workload
            # (untimed warm-up work), keep the faster for the timed views
            # (interleaved: 3 rounds of 8 views per candidate, ~0.2 s)
            self.tuned = {k: 0.0 for k in self.cands}
            n_tune, rounds = 8, 3
            # the shader clock of each tuning group too (the timed views'
            # clock is beside it in the line: a box whose clock moved between
            # the tuning and the timed views shows it)
            tstamps = torch.zeros(rounds * len(self.cands), 2, 768, dtype=torch.int64, device=self.dev)
            cur = torch.cuda.current_stream(self.dev)
            for rnd in range(rounds):
                for ci, k in enumerate(self.cands):
                    self.n_active, self.n_step = k, 0
                    torch.cuda.synchronize()
                    if self.world > 1:
                        dist.barrier()
                    t0 = time.perf_counter()
                    sg = tstamps[rnd * len(self.cands) + ci]
                    lib().samnerf_clock_stamp(ctypes.c_void_p(sg[0].data_ptr()), ctypes.c_void_p(cur.cuda_stream))
                    for _ in range(n_tune):
                        self.step()
                    self._flush()
                    for st in self.streams:
                        if st.cuda_stream != cur.cuda_stream:
                            cur.wait_stream(st)
                    lib().samnerf_clock_stamp(ctypes.c_void_p(sg[1].data_ptr()), ctypes.c_void_p(cur.cuda_stream))
                    torch.cuda.synchronize()
                    dtk = time.perf_counter() - t0
                    if self.world > 1:
                        tk = torch.tensor([dtk], device=self.dev if self.args.dist_backend == "nccl" else "cpu")
                        dist.all_reduce(tk, op=dist.ReduceOp.MAX)
                        dtk = tk.item()
                    self.tuned[k] += dtk * 1e3 / (n_tune * rounds)
            self.n_active = min(self.tuned, key=self.tuned.get)
            self.n_step = 0
            ts = tstamps.cpu().numpy()
            self.tuned_clock = {}
            for ci, k in enumerate(self.cands):
                g = [timed_clock(ts[rnd * len(self.cands) + ci]) for rnd in range(rounds)]
                g = [c["ghz"] for c in g if c]
                self.tuned_clock[k] = float(np.mean(g)) if g else None
        stamps = torch.zeros(2, 768, dtype=torch.int64, device=self.dev)
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # the shader clock of the timed views: one stamp before the first and
        # one after the last (the current stream waits for the others first)
        lib().samnerf_clock_stamp(ctypes.c_void_p(stamps[0].data_ptr()),
                                  ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream))
        last = None
        for i in range(steps):
            last = self.step()                   # no stage events in the timed views (below)
        flushed = self._flush()                  # the last view's gather is inside the timed region
        cur = torch.cuda.current_stream(self.dev)
        for st in self.streams:
            if st.cuda_stream != cur.cuda_stream:
                cur.wait_stream(st)
        lib().samnerf_clock_stamp(ctypes.c_void_p(stamps[1].data_ptr()), ctypes.c_void_p(cur.cuda_stream))
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        lib().samnerf_set_stage_events(None, 0)
        self.clock = timed_clock(stamps.cpu().numpy())
        if flushed:
            last = flushed[-1]
        if self.world > 1:
            t = torch.tensor([dt], device=self.dev if self.args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = t.item()
        if not stages:
            return dt, last, None, None
        # Stage times for the rooflines from a single-stream pass after the
        # timed region: with several views in flight, one view's HIP events
        # also span the other streams' kernels, and the timed views carry no
        # per-stage event records at all (round 6).  Every rank runs it (the
        # views' gathers are collectives).
        n_roof = min(steps, 5)
        sets = [[make_event_set() for _ in range(self.chunks)] for _ in range(n_roof)]
        torch.cuda.synchronize()
        for i in range(n_roof):
            self._step_on_stream([raw for _, raw in sets[i]])
        self._flush()
        torch.cuda.synchronize()
        lib().samnerf_set_stage_events(None, 0)
        stage_src = f"a single-stream pass of {n_roof} views after the timed region"
        stage_avg = {}          # per step: summed over the chunks of the rank's band
        for j, st in enumerate(STAGES):
            stage_avg[st] = float(np.mean([sum(evs[j].elapsed_time(evs[j + 1]) for evs, _ in chunk_sets)
                                           for chunk_sets in sets]))
        return dt, last, stage_avg, stage_src


def timed_clock(stamps):
    """Shader clock of the timed views from two samnerf_clock_stamp records
    (256 workgroups each: XCC id, s_memtime, s_memrealtime): per XCD the
    median tick counts at each end, clock = d(memtime) / d(memrealtime) x
    100 MHz; the mean over the XCDs seen at both ends."""
    a, b = stamps[0].reshape(256, 3), stamps[1].reshape(256, 3)
    per = {}
    for x in sorted(set(a[:, 0].tolist()) & set(b[:, 0].tolist())):
        ta, tb = a[a[:, 0] == x], b[b[:, 0] == x]
        dt = float(np.median(tb[:, 1]) - np.median(ta[:, 1]))
        dr = float(np.median(tb[:, 2]) - np.median(ta[:, 2]))
        if dr > 0:
            per[int(x)] = dt / dr * 0.1                 # GHz (s_memrealtime: 100 MHz)
    if not per:
        return None
    return {"ghz": float(np.mean(list(per.values()))), "per_xcd_ghz": {str(k): round(v, 4) for k, v in per.items()},
            "what": "shader clock over the timed views: s_memtime ticks / s_memrealtime (100 MHz) between "
                    "two samnerf_clock_stamp launches bracketing them (median per XCD, mean over XCDs)"}


def explain_gather(runner, views=5):
    """N > 1: what one view costs each rank, measured apart so the driver's
    scaling run explains itself.  Per view: the band's
    render (HIP events on the render stream around samnerf_render_forward_tile
    into this rank's slice of the gather buffer) and then the all-gather alone
    (RCCL: all_gather_into_tensor, the current stream waiting on the
    collective's stream; events on the current stream around it), not
    overlapped, so gather_ms / render_ms says which of the two the pipelined
    timing is bound by.  Bytes: what each rank receives per view.  Returns
    rank 0's record (all ranks take part)."""
    from samnerf_amd.dist import _all_gather
    args, dev, H, W = runner.args, runner.dev, runner.H, runner.W
    from samnerf_amd import ops
    ro, rd = ops.get_rays(runner.pose, runner.intr, H, W, device=dev, row0=runner.r0, rows=runner.r1 - runner.r0)
    n = ro.shape[0]
    cols = 5 if args.no_sam else 261
    buf = torch.empty(runner.world * n, cols, device=dev)
    own = buf[dist.get_rank() * n:(dist.get_rank() + 1) * n]
    rms, gms = [], []
    for i in range(views + 1):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda.synchronize()
        e0.record()
        runner.renderer.render(ro, rd, view_width=W if args.tiles else 0, out_tile=own)
        e1.record()
        _all_gather(buf, own, None, async_op=False)
        e2.record()
        torch.cuda.synchronize()
        if i:                                            # the first view warms the collective
            rms.append(e0.elapsed_time(e1))
            gms.append(e1.elapsed_time(e2))
    mine = torch.tensor([float(np.mean(rms)), float(np.mean(gms))], dtype=torch.float64)
    allr = [torch.zeros(2, dtype=torch.float64) for _ in range(runner.world)]
    if args.dist_backend == "nccl":
        g = [t.to(dev) for t in allr]
        dist.all_gather(g, mine.to(dev))
        allr = [t.cpu() for t in g]
    else:
        dist.all_gather(allr, mine)
    render = [float(t[0]) for t in allr]
    gather = [float(t[1]) for t in allr]
    recv = (runner.world - 1) * n * cols * 4
    return {"per_rank_render_ms": render, "per_rank_gather_ms": gather,
            "bytes_received_per_rank_per_view": recv,
            "gather_GBps_per_rank": recv / (max(gather) * 1e-3) / 1e9,
            "gather_over_render": max(gather) / (sum(render) / len(render)),
            "views": views, "backend": args.dist_backend,
            "what": "each rank renders its band into its slice of the gather buffer, then the all-gather "
                    "runs alone (not overlapped): render_ms = HIP events on the render stream, gather_ms = "
                    "events on the current stream around all_gather_into_tensor (waits for RCCL's stream); "
                    "the timed headline overlaps view i's gather with view i+1's render, so a view costs "
                    "about max(render, gather) when gather_over_render < 1"}


VALU_RATE = os.path.join(REPO, "profiles", "r4_valu_rate.json")
# per-stage issue cycles per VALU instruction: the stage kernel's opcode mix x
# the measured per-opcode rates (tools/valu_cpi.py, round 5)
VALU_CPI = os.path.join(REPO, "profiles", "r6_valu_cpi.json")


def valu_cpi_of_stages():
    try:
        return {k: v["cycles_per_inst"] for k, v in json.load(open(VALU_CPI))["stages"].items()}
    except Exception:
        return {}


def valu_cycles_per_inst():
    """Cycles per wave64 VALU instruction of one SIMD at saturation, measured
    by tools/valu_rate.hip (profiles/r4_valu_rate.json: independent v_fma_f32
    streams, the best over 1-8 resident waves per SIMD); the guide's 2 cycles
    (MI355X_MICROARCH.md, SIMD-32) without the file."""
    try:
        r = json.load(open(VALU_RATE))["kinds"]["v_fma_f32"]
        return min(v["cycles_per_inst"] for v in r.values()), os.path.relpath(VALU_RATE, REPO)
    except Exception:
        return 2.0, "MI355X_MICROARCH.md (2 cycles per v_fma_f32, SIMD-32)"


def rooflines(stage_avg, band_rays, head_mode, rates, clocks=None, timed_clock=None):
    """`roofline` of the dominant kernel and every stage, each against the
    guide peak of its units:
      l2   -- algorithmic bytes (embedding gathers + ray I/O, ALG_BYTES_PER_RAY)
              / live time vs the L2's 34.5 TB/s (the tables are L2/MALL-resident;
              not for s_grid, whose box gathers read a row once per wave);
      valu -- the VALU pipe's share: issued VALU instructions (PMC SQ_INSTS_VALU
              per ray, profiles/pmc_rates.json) x the stage kernel's issue
              cycles per instruction (profiles/r6_valu_cpi.json: its opcode
              mix priced at the measured per-opcode rates, 3.5-3.75; without
              the file the v_fma_f32 rate, 2.2) / (1024 SIMDs x 2.4 GHz x
              live time);
      mfma -- MFMA-busy cycles (PMC SQ_VALU_MFMA_BUSY_CYCLES per ray) over the
              same SIMD cycles; for the SAM head also from its structure (86
              k-blocks x 8 tiles x 3 v_mfma_f32_32x32x16_f16 per 32 rays).
    `bound` is the unit with the largest share; when none reaches 0.6 the stage
    is marked latency-bound (`regime`), with the PMC wave-cycle shares --
    waiting on memory / barriers, issue stalls, issuing -- beside it.  The nominal clock makes every share a lower
    bound; `frac_at_measured_clock` rescales by the stage's measured clock
    (profiles/kernel_clock.json)."""
    st_rates = (rates or {}).get("stages", {})
    cyc_avail = lambda ms: N_SIMD * CLOCK_GHZ * 1e9 * ms * 1e-3
    cpi, cpi_src = valu_cycles_per_inst()
    stage_cpi = valu_cpi_of_stages()

    def entry(st):
        ms = stage_avg.get(st, 0.0)
        if ms <= 0:
            return None
        r = st_rates.get(st, {})
        alg = ALG_BYTES_PER_RAY[st] * band_rays
        cand = {}
        if st != "s_grid":
            cand["l2"] = {"unit": "GB/s", "achieved": alg / (ms * 1e-3) / 1e9, "peak": L2_PEAK_GBS,
                          "alg_bytes_per_ray": ALG_BYTES_PER_RAY[st]}
            cand["l2"]["frac"] = cand["l2"]["achieved"] / L2_PEAK_GBS
        if "valu_insts_per_ray" in r:
            ci, ci_src = (stage_cpi[st], os.path.relpath(VALU_CPI, REPO)) if st in stage_cpi else (cpi, cpi_src)
            c = r["valu_insts_per_ray"] * band_rays * ci
            cand["valu"] = {"unit": "VALU-busy cycles per SIMD per ns (GHz); peak = the nominal clock",
                            "frac": c / cyc_avail(ms),
                            "valu_insts_per_ray": r["valu_insts_per_ray"], "cycles_per_inst": ci,
                            "cycles_per_inst_source": ci_src,
                            # the other basis: every VALU
                            # instruction at the measured v_fma_f32 rate
                            "frac_fma_rate_basis": r["valu_insts_per_ray"] * band_rays * cpi / cyc_avail(ms),
                            "fma_rate_cycles_per_inst": cpi, "fma_rate_source": cpi_src}
            if "valu_cycles_per_ray" in r:
                # the counter's VALU cycles: SQ_ACTIVE_INST_VALU
                # x 4 (quad-cycles each wave spends on VALU instructions; the
                # basis of AMD's derived VALUBusy = 100 SQ_ACTIVE_INST_VALU /
                # CU_NUM / GRBM_GUI_ACTIVE, rocprofiler-sdk counter_defs.yaml),
                # against the static opcode-mix estimate; beyond 10 % apart the
                # line takes the counter.  (SQ_THREAD_CYCLES_VALU / 64, the
                # other gfx950 VALU counter, is ~1.0 per instruction: it counts
                # lane-instructions, not issue cycles -- profiles/r6c_valu_counters.txt.)
                pc = r["valu_cycles_per_ray"] * band_rays
                v = cand["valu"]
                v["pmc_cycles_per_inst"] = r["valu_cycles_per_ray"] / r["valu_insts_per_ray"]
                v["frac_pmc"] = pc / cyc_avail(ms)
                v["static_over_pmc"] = c / pc if pc > 0 else None
                if pc > 0 and abs(c / pc - 1.0) > 0.10:
                    v["frac_static_opcode_mix"] = v["frac"]
                    v["frac"] = v["frac_pmc"]
                    v["basis"] = ("PMC: SQ_ACTIVE_INST_VALU x 4 (VALUBusy); the static opcode-mix estimate is "
                                  "more than 10 % below it")
                else:
                    v["basis"] = "static opcode mix, within 10 % of PMC SQ_ACTIVE_INST_VALU x 4"
            # achieved / peak in the unit: VALU-busy cycles per SIMD per ns
            # against the SIMD's nominal 2.4 cycles per ns (frac = their ratio)
            cand["valu"]["achieved"] = cand["valu"]["frac"] * CLOCK_GHZ
            cand["valu"]["peak"] = CLOCK_GHZ
        if st == "sam_head":
            cyc = HEAD_MFMA_CYCLES_PER_32[head_mode] * band_rays / 32
            cand["mfma"] = {"unit": "TFLOP/s", "frac": cyc / cyc_avail(ms),
                            "achieved_fp32_equiv": HEAD_FLOP_PER_RAY * band_rays / (ms * 1e-3) / 1e12,
                            "peak": F32_MFMA_PEAK_TFS if head_mode == 1 else BF16_MFMA_PEAK_TFS,
                            "achieved": None,
                            "basis": "MFMA issue cycles of the head's structure (f16x3, k_sam_head_w8: 44 "
                                     "32-deep k-blocks x 16 tiles x 3 v_mfma_f32_16x16x32_f16 per 16 rays) / "
                                     "(1024 SIMDs x 2.4 GHz x time)"}
            cand["mfma"]["achieved"] = cand["mfma"]["frac"] * cand["mfma"]["peak"]   # at the structure's rate
            if "mfma_busy_cycles_per_ray" in r:
                cand["mfma"]["pmc_mfma_busy_frac"] = r["mfma_busy_cycles_per_ray"] * band_rays / cyc_avail(ms)
        elif r.get("mfma_busy_cycles_per_ray"):
            f = r["mfma_busy_cycles_per_ray"] * band_rays / cyc_avail(ms)
            cand["mfma"] = {"unit": "MFMA-busy cycles per SIMD per ns (GHz); peak = the nominal clock",
                            "frac": f, "achieved": f * CLOCK_GHZ, "peak": CLOCK_GHZ}
        if not cand:
            return None
        bound = max(cand, key=lambda k: cand[k]["frac"])
        e = {"bound": bound}
        if cand[bound]["frac"] < 0.6:
            e["regime"] = "latency-bound: no unit reaches 0.6 of its peak (wave_cycle_shares)"
        if "wave_cycle_shares" in r:
            e["wave_cycle_shares"] = r["wave_cycle_shares"]
        if st == "s_grid":
            # the box form reads each distinct corner row once per wave, so the
            # algorithmic gather bytes (every lane's 8 corners) are no traffic
            # bound: reported, not priced
            e["alg_gather_tbs"] = alg / (ms * 1e-3) / 1e12
        e.update(cand[bound])
        e["other_bounds"] = {k: v["frac"] for k, v in cand.items() if k != bound}
        clk = (clocks or {}).get("stages", {}).get(st)
        if clk and bound in ("valu", "mfma"):
            # the same busy cycles over the cycles the stage had at the clock it
            # ran at (profiles/kernel_clock.json, tools/kernel_clock.py)
            e["measured_clock_ghz"] = clk
            e["frac_at_measured_clock"] = e["frac"] * CLOCK_GHZ / clk
        if timed_clock and bound in ("valu", "mfma"):
            # at the clock measured live over this run's timed views
            e["timed_clock_ghz"] = timed_clock["ghz"]
            e["frac_at_timed_clock"] = e["frac"] * CLOCK_GHZ / timed_clock["ghz"]
            if "frac_fma_rate_basis" in e:
                e["frac_fma_rate_basis_at_timed_clock"] = e["frac_fma_rate_basis"] * CLOCK_GHZ / timed_clock["ghz"]
        if "ta_busy_frac_in_pmc_run" in r:
            e["ta_busy_frac_in_pmc_run"] = r["ta_busy_frac_in_pmc_run"]
        return e

    stages = {st: entry(st) for st in STAGES}
    stages = {k: v for k, v in stages.items() if v is not None}
    cands = {k: stage_avg[k] for k in STAGES if stage_avg.get(k, 0) > 0}
    dom = max(cands, key=cands.get)
    roof = dict(stages[dom])
    roof.update({"kernel": dom, "avg_launch_ms": stage_avg[dom],
                 "alg_bytes_per_launch": ALG_BYTES_PER_RAY[dom] * band_rays})
    hb = st_rates.get(dom, {}).get("hbm_bytes_per_ray")
    t = hb * band_rays if hb else None
    roof["traffic"] = t
    roof["hbm_frac_counters"] = (t / (stage_avg[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS) if t else None
    roof["pmc_source"] = os.path.relpath(PMC_RATES, REPO) if rates else None
    return roof, stages


def pmc_rates():
    """profiles/pmc_rates.json (tools/pmc_rates.py), or None."""
    try:
        return json.load(open(PMC_RATES))
    except Exception:
        return None


def stage_clocks():
    """profiles/kernel_clock.json (tools/kernel_clock.py --json), or None."""
    try:
        return json.load(open(os.path.join(REPO, "profiles", "kernel_clock.json")))
    except Exception:
        return None


def main():
    args = parse()
    rc = maybe_launch(args)
    if rc is not None:
        sys.exit(rc)
    if args.mode in ("train", "gui", "rgbtrain"):
        if args.gpus != 1:
            raise SystemExit(f"--mode {args.mode} runs on one GPU")
        torch.cuda.set_device(0)
        fn = {"train": train_main, "gui": gui_main, "rgbtrain": rgb_train_main}[args.mode]
        return fn(args, torch.device("cuda", 0))
    rank, world, dev = setup_dist(args)
    from samnerf_amd import ops
    from samnerf_amd.dist import shard_range
    from samnerf_amd.fused import FusedRenderer
    from samnerf_amd import synth

    with_sam = not args.no_sam
    net, spec, params = build_net(with_sam, dev, seed=3 if args.scene == "surface" else 0,
                                  surface=args.scene == "surface")
    renderer = FusedRenderer(net, head_mode=args.head_mode)
    H, W = args.H, args.W
    pose, intr = synth.gui_camera(W, H)
    r0, r1 = shard_range(H, rank, world)                      # row band of this rank
    n_total = H * W
    if world == 1 and args.rank_share > 1:                     # one rank's band, on one GPU
        k = args.share_rank if args.share_rank >= 0 else args.rank_share // 2
        r0, r1 = shard_range(H, k, args.rank_share)
        n_total = (r1 - r0) * W
    band_rays = (r1 - r0) * W
    codec = args.gather_codec

    runner = ViewRunner(args, renderer, world, dev, H, W, pose, intr, r0, r1, codec)
    dt, last, stage_avg, stage_src = runner.run(args.steps, args.warmup)
    value = n_total * args.steps / dt
    roof, stage_roof = rooflines(stage_avg, band_rays, args.head_mode, pmc_rates(), stage_clocks(),
                                 runner.clock)

    side = {}
    if world > 1 and args.chunks == 0 and codec == "fp32":
        side["gather_explained"] = explain_gather(runner)
    if not args.no_alt and world > 1 and with_sam and args.chunks == 0:
        # the other transport, same views, after the headline
        other = "q16" if codec == "fp32" else "fp32"
        r2 = ViewRunner(args, renderer, world, dev, H, W, pose, intr, r0, r1, other)
        dt2, last2, _, _ = r2.run(args.steps, args.warmup, stages=False)
        err = (last2["samvit"] - last["samvit"]).abs().max().reshape(1).float()
        if args.dist_backend != "nccl":
            err = err.cpu()
        dist.all_reduce(err, op=dist.ReduceOp.MAX)
        side[f"gather_codec_{other}"] = {
            "value": n_total * args.steps / dt2, "unit": "rays/s", "ms_per_step": dt2 * 1e3 / args.steps,
            "max_abs_samvit_vs_" + codec: float(err.item()),
            "what": "q16: 536 B/ray transport, samvit int16 x per-ray power-of-two scale, |err| <= "
                    "2^-14 of the ray's max |samvit|, own band fp32" if other == "q16" else
                    "fp32: 1,044 B/ray exact transport"}
    if not args.no_alt and world == 1 and args.rank_share <= 1:
        # the other precision mode on the same view (DTYPE)
        other = 1 - args.head_mode
        r3 = ViewRunner(args, FusedRenderer(net, head_mode=other), 1, dev, H, W, pose, intr, r0, r1, codec)
        dt3, last3, st3, _ = r3.run(max(3, args.steps // 2), 2)
        side["precision_" + ("exact_fp32" if other == 1 else "f16x3")] = {
            "value": n_total * max(3, args.steps // 2) / dt3, "unit": "rays/s",
            "ms_per_step": dt3 * 1e3 / max(3, args.steps // 2), "stage_ms": st3, "dtype": DTYPE[other],
            "max_abs_samvit_vs_headline": float((last3["samvit"] - last["samvit"]).abs().max())
            if with_sam else None,
            "max_abs_image_vs_headline": float((last3["image"] - last["image"]).abs().max())}

    if not args.no_alt and world == 1 and args.rank_share <= 1:
        # N1, the flagged non-parity early exit (samnerf_model.t_thresh), on a
        # scene whose rays saturate (random weights never do); timed against
        # the default mode on the same scene and view
        snet, _, _ = build_net(with_sam, dev, seed=3, surface=True)
        k = max(3, args.steps // 2)
        n1 = {}
        for t in (0.0, 1e-4):
            rn = ViewRunner(args, FusedRenderer(snet, head_mode=args.head_mode, t_thresh=t), 1, dev,
                            H, W, pose, intr, r0, r1, codec)
            dtn, lastn, stn, _ = rn.run(k, 2)
            n1[t] = (dtn, lastn, stn, rn.n_active, rn.tuned)
        base, fast = n1[0.0], n1[1e-4]
        # the trained-scene regime (proposal samples concentrated at a surface)
        # in the default mode: the headline's configuration on another scene
        side["surface_scene"] = {
            "value": n_total * k / base[0], "unit": "rays/s", "ms_per_step": base[0] * 1e3 / k,
            "stage_ms": base[2], "vs_headline_ms": (base[0] * 1e3 / k) / (dt * 1e3 / args.steps),
            "streams": base[3], "streams_tuned_ms": base[4],
            "what": "the headline configuration (cfg3) on the opaque-sphere scene "
                    "(synth.make_surface_params: a trained scene's regime, samples at the surface), "
                    "default mode (reference semantics)"}
        err_n1 = float((base[1]["samvit"] - fast[1]["samvit"]).abs().max()) if with_sam else 0.0
        side["n1_early_exit"] = {
            "value": n_total * k / fast[0], "unit": "rays/s", "ms_per_step": fast[0] * 1e3 / k,
            "default_mode_ms_per_step": base[0] * 1e3 / k, "speedup": base[0] / fast[0],
            "t_thresh": 1e-4, "stage_ms": fast[2], "default_mode_stage_ms": base[2],
            "max_weights_sum_drop": float((base[1]["weights_sum"] - fast[1]["weights_sum"]).max()),
            "max_abs_image_vs_default": float((base[1]["image"] - fast[1]["image"]).abs().max()),
            **({"max_abs_samvit_vs_default": float((base[1]["samvit"] - fast[1]["samvit"]).abs().max())}
               if with_sam else {}),
            "exceeds_1e-3_bar": err_n1 > 1e-3 or
                                float((base[1]["image"] - fast[1]["image"]).abs().max()) > 1e-3,
            "what": "FLAGGED NON-PARITY mode (SURVEY H6), never the default: a wave of 32 rays stops the "
                    "final stage once every ray's transmittance < t_thresh; opaque-sphere scene "
                    "(synth.make_surface_params), same view; its output error against the default "
                    "mode is reported above and, where exceeds_1e-3_bar is true, breaks the "
                    "north star's 1e-3 feature bar"}

    if not args.no_alt and world == 1 and args.rank_share <= 1 and with_sam:
        # BASELINE config 2 (512x512 RGB only; renderer.py:221-362 without the
        # SAM branch) on the same view: its own model, the fused path and the
        # reference's op sequence on the same GPU
        rnet, _, _ = build_net(False, dev)
        k = max(3, args.steps // 2)
        r2 = ViewRunner(args, FusedRenderer(rnet, head_mode=args.head_mode), 1, dev, H, W, pose, intr,
                        r0, r1, codec)
        dt2, _, st2, _ = r2.run(k, 2)
        ref2 = None
        if args.ref_gpu_rays:
            ro2, rd2 = ops.get_rays(pose, intr, H, W, device=dev)
            ref2 = reference_equivalent_gpu(rnet, ro2, rd2, min(args.ref_gpu_rays, 65536))
        side["cfg2_rgb"] = {
            "value": n_total * k / dt2, "unit": "rays/s", "ms_per_step": dt2 * 1e3 / k, "steps": k,
            "stage_ms": {kk: v for kk, v in st2.items() if kk in ("prop0", "prop1", "final")},
            "reference_equivalent_gpu": ref2,
            "speedup": (n_total * k / dt2) / ref2["value"] if ref2 else None,
            "what": "BASELINE cfg2: 512x512 RGB-only model (with_sam=False), same camera; parity: "
                    "tests/test_gpu_fullview.py[cfg2_rgb] (every ray vs the oracle)"}
        # the GUI's frame (readme.md:5's 5 FPS includes the SAM decoder)
        dtg = gui_frame_time(dev, H, W, max(3, args.steps // 2), 2, net=net)
        side["gui_frame"] = {
            "value": 1.0 / dtg, "unit": "frames/s", "ms_per_step": dtg * 1e3,
            "rays_per_s": (H * W + 64 * 64) / dtg,
            "what": f"GUI frame (nerf/gui.py:143-161, utils.py:1647-1712): {H}x{W} RGB (features "
                    "skipped, return_feats=0) + 64x64 rays with 256-d SAM features; readme.md:5 quotes "
                    "5 FPS on a V100 for this loop including the SAM decoder (not run here)"}

    if not args.no_alt and world == 1 and args.rank_share <= 1:
        # perturb=True (renderer.py:266-271, :100-101: the distillation step's
        # teacher render, the GUI's spp > 1) on the fused kernels, the torch
        # draws of the perturbed positions inside the timed region
        fr = FusedRenderer(net, head_mode=args.head_mode)
        ro, rd = ops.get_rays(pose, intr, H, W, device=dev)
        k = max(3, args.steps // 2)
        for _ in range(2):
            outp = fr.render(ro, rd, feats=with_sam, view_width=W, perturb=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            outp = fr.render(ro, rd, feats=with_sam, view_width=W, perturb=True)
        torch.cuda.synchronize()
        dtp = (time.perf_counter() - t0) / k
        side["perturbed_render"] = {
            "value": H * W / dtp, "unit": "rays/s", "ms_per_step": dtp * 1e3, "steps": k,
            "max_abs_image_vs_unperturbed": float((outp["image"] - last["image"]).abs().max()),
            "what": "the headline view with perturb=True: torch.rand_like draws of the perturbed "
                    "stage-0 bins and sample_pdf positions (fused.perturbed_positions) + the fused "
                    "render fed them (samnerf_model.perturb), one stream"}

    if not args.no_alt and world == 1 and args.rank_share <= 1:
        # the --with_mask instance head on the fused kernels
        side["mask_default_head"] = mask_view(dev, max(3, args.steps // 2), 2, args.head_mode)

    if not args.no_alt and world == 1 and args.rank_share <= 1 and with_sam:
        # BASELINE config 5 beside the headline (`--mode train` runs it alone)
        ms5, loss5 = train_steps(dev, 20, 5)
        ms5d, loss5d = train_steps(dev, 20, 5, deterministic=True)
        side["cfg5_train"] = {"ms_per_step": ms5, "steps_per_s": 1e3 / ms5,
                              "rays_per_s": 4096 * 1e3 / ms5, "steps": 20, "warmup": 5,
                              "final_loss": loss5, **TRAIN_WHAT,
                              "deterministic_mode": {
                                  "ms_per_step": ms5d, "final_loss": loss5d,
                                  "what": "the same steps with the s_grid scatter in 64-bit fixed point "
                                          "(samnerf_sgrid_backward_det, SURVEY H5): gradients repeat bit for "
                                          "bit (tests/test_gpu_train.py::test_distillation_steps_repeat_bit_for_bit)"}}

    if not args.no_alt and world == 1 and args.rank_share <= 1:
        # the reference's RGB training stage on the HIP training
        # kernels, the torch path beside it
        msr, lossr = rgb_train_steps(dev, 20, 5, fused=True)
        msr_t, _ = rgb_train_steps(dev, 6, 2, fused=False)
        side["rgb_train"] = {"ms_per_step": msr, "steps_per_s": 1e3 / msr, "rays_per_s": 8192 * 1e3 / msr,
                             "steps": 20, "warmup": 5, "final_loss": lossr,
                             "torch_path_ms_per_step": msr_t, "speedup_vs_torch_path": msr_t / msr,
                             **RGB_TRAIN_WHAT}

    if not args.no_alt and world == 1 and args.rank_share <= 1:
        # the --with_mask training step on the HIP mask-training
        # kernels, the torch path beside it
        msm, lossm = mask_train_steps(dev, 20, 5, fused=True)
        msm_t, _ = mask_train_steps(dev, 6, 2, fused=False)
        side["mask_train"] = {
            "ms_per_step": msm, "steps_per_s": 1e3 / msm, "rays_per_s": 4096 * 1e3 / msm, "steps": 20,
            "warmup": 5, "final_loss": lossm, "torch_path_ms_per_step": msm_t,
            "speedup_vs_torch_path": msm_t / msm,
            "dtype": "fp32 (render forward in the fused op order; mask head forward + backward on exact "
                     "fp32 MFMA, mask_head_train.hip; m_grid scatter and dW by fp32 atomics)",
            "what": "--with_mask training step (utils.py:941-977): 4096 rays at random pixels of a 512x512 "
                    "view, 'default' head (m_grid L16C8 2^19 + SkipConnMLP 143->256->256->2), softmax / "
                    "clamp / NLL, backward, Adam over m_grid + mask_mlp"}

    if rank == 0:
        rec = {
            "metric": METRIC, "value": value, "unit": "rays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt * 1e3 / args.steps,
            "streams": runner.n_active,
            "streams_tuned_ms": runner.tuned,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": DTYPE[args.head_mode],
            "data": ("synthetic (random-init weights of the reference architecture, GUI camera)"
                     if args.scene == "default" else
                     "synthetic opaque-sphere scene (synth.make_surface_params), GUI camera"),
            "config": {"workload": ("cfg3: 512x512 view, RGB + 256-d SAM feature per ray" if with_sam
                                    else "cfg2: 512x512 view, RGB only") if (H, W) == (512, 512)
                       else f"{H}x{W} view", **({"rank_share": f"rows {r0}-{r1} of {args.rank_share} bands"}
                                                 if world == 1 and args.rank_share > 1 else {}),
                       "rays_per_step": n_total, "num_steps": [128, 64, 32],
                       # how the timed views ran: views in
                       # flight (HIP streams) the warm-up tuner chose, its
                       # per-candidate ms per view, and the shader clock
                       # measured over the timed views
                       "views_in_flight": runner.n_active,
                       "views_in_flight_tuned_ms": ({str(k): round(v, 4) for k, v in runner.tuned.items()}
                                                    if runner.tuned else None),
                       "views_in_flight_tuned_clock_ghz": ({str(k): (round(v, 4) if v else None)
                                                            for k, v in runner.tuned_clock.items()}
                                                           if runner.tuned_clock else None),
                       "timed_clock_ghz": round(runner.clock["ghz"], 4) if runner.clock else None,
                       "parallelism": (f"ray-sharded row bands x{world}, RCCL all-gather of each view "
                                       f"overlapped with the next view's rendering, views issued on "
                                       f"{runner.n_active} HIP streams" if args.chunks == 0 else
                                       f"ray-sharded row bands x{world}, {runner.chunks} chunks per band, "
                                       "async RCCL all-gather per chunk") if world > 1
                       else "single GPU",
                       **({"gather_codec": codec + (" (536 B/ray: samvit int16 x per-ray power-of-two "
                                                    "scale, |err| <= 2^-14 of the ray max; own band fp32)"
                                                    if codec == "q16" else " (1,044 B/ray, exact)")}
                          if world > 1 and args.chunks == 0 else {})},
            "timed_clock": runner.clock,
            "stage_ms_source": stage_src,
            "roofline": roof,
            "stage_ms": stage_avg,
            "stage_roofline": stage_roof,
            **side,
        }
        if world == 1 and args.ref_gpu_rays > 0:
            ro_all, rd_all = ops.get_rays(pose, intr, H, W, device=dev)
            ref = reference_equivalent_gpu(net, ro_all, rd_all, args.ref_gpu_rays)
            ref["speedup"] = value / ref["value"]
            rec["reference_equivalent_gpu"] = ref
        if world == 1 and args.cpu_rays > 0:
            # parity weights (embeddings U(+-0.5)): a non-trivial
            # scene for the PSNR / max-error comparison; the same view
            pnet, pspec, pparams = build_net(with_sam, dev, seed=33, emb_scale=0.5)
            ro_all, rd_all = ops.get_rays(pose, intr, H, W, device=dev)
            pout = FusedRenderer(pnet, head_mode=args.head_mode).render(ro_all, rd_all)
            torch.cuda.synchronize()
            rec["cpu_baseline"], rec["parity_vs_ref"] = cpu_baseline(
                pspec, pparams, pose, intr, H, W, args.cpu_rays, gpu_out=pout)
        else:
            rec["cpu_baseline"] = None
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
