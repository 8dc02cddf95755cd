"""SAM-feature distillation step (BASELINE config 5) on the MI355X.

The fused forward + HIP s_grid scatter must give the same gradients as the
reference's unfused autograd graph (run_torch: torch ops + drop-in grid
backward kernel), and a few Adam steps must reduce the loss
(nerf/utils.py:1072-1106, main.py:255-262, :296).
"""
import pytest
import torch
import torch.nn.functional as F

from helpers import make_net
from oracle import synth

pytestmark = pytest.mark.gpu


def _frozen_net(cuda, seed=5):
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    params = synth.make_params(spec, seed=seed, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    for k, p in net.named_parameters():          # main.py:255-262: RGB params frozen
        p.requires_grad = k.startswith("s_grid") or k.startswith("samvit_mlp")
    return net


def test_fused_sgrid_backward_matches_autograd(hip_lib, cuda):
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, render_sam_train
    net = _frozen_net(cuda)
    net.train()
    pose, intr = synth.gui_camera(32, 32, rot=synth.random_rotation(8))
    ro, rd = ops.get_rays(pose, intr, 32, 32, device=cuda)
    G = torch.randn(32 * 32, 256, device=cuda)

    from oracle_backend import injected_bins
    out = render_sam_train(FusedRenderer(net), ro, rd)
    (out["samvit"] * G).sum().backward()
    g_fused = {k: p.grad.clone() for k, p in net.named_parameters() if p.requires_grad}
    net.zero_grad(set_to_none=True)
    taps = FusedRenderer(net).render(ro, rd, taps=True)       # the fused path's resampled bins

    with injected_bins([taps["bins1"].contiguous(), taps["bins2"].contiguous()]):
        ref = net.run_torch(ro, rd, return_feats=1)
    (ref["samvit"] * G).sum().backward()
    g_ref = {k: p.grad.clone() for k, p in net.named_parameters() if p.requires_grad}
    assert torch.allclose(out["samvit"], ref["samvit"], atol=1e-3)
    for k in g_ref:
        a, b = g_fused[k], g_ref[k]
        err = (a - b).abs().max().item()
        scale = b.abs().max().item()
        assert err <= 2e-3 * max(scale, 1e-3), f"{k}: {err} vs scale {scale}"


@pytest.mark.parametrize("det", [False, True])
def test_distillation_step_matches_cpu_twin_full_tables(hip_lib, cuda, det):
    """BASELINE config 5 at the reference's table sizes (s_grid 2^19 rows per
    hashed level, 5,258,512 rows x 8; 4096 rays of a 64x64 camera): the fused
    forward + HIP s_grid scatter + head backward on the GPU against the
    reference's op sequence on the CPU (the mirror's run_torch with the C
    oracle's encoder forward / backward: tests/oracle_backend.py), the same
    loss (utils.py:1098-1106: bilinear resize + MSE vs an N(0,1) target).
    Loss to fp32 rounding; at the same resampled bins, gradients of
    s_grid.embeddings and every samvit_mlp tensor within 1e-4 relative (norm):
    float atomics, GPU vs CPU GEMM order, f16x3 grid_mlp forward
    (fp32-equivalent).  det: the s_grid scatter in the deterministic mode
    (samnerf_sgrid_backward_det, 64-bit fixed point)."""
    from oracle import renderer as orc
    from oracle_backend import injected_bins, oracle_encoders
    from samnerf_amd.fused import FusedRenderer
    from samnerf_amd.train import sam_train_step
    spec = synth.ModelSpec(with_sam=True)                      # 19 / 19 / 17, as network.py
    params = synth.make_params(spec, seed=7, emb_scale=0.5, ln_jitter=0.1)
    nets = {"gpu": make_net(spec, params, cuda), "cpu": make_net(spec, params, "cpu")}
    for net in nets.values():
        net.train()
        for k, p in net.named_parameters():                    # main.py:255-262
            p.requires_grad = k.startswith("s_grid") or k.startswith("samvit_mlp")
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(10))
    ro, rd = orc.get_rays(pose, intr, 64, 64)
    gt = torch.randn(1, 256, 64, 64, generator=torch.Generator().manual_seed(1))
    _, lg = sam_train_step(FusedRenderer(nets["gpu"], deterministic=det), ro.to(cuda), rd.to(cuda), 64, 64,
                           gt.to(cuda))
    lg.backward()
    # the twin samples at the fused path's resampled bins (an ulp of a sample
    # position moves the fine levels' gradients: tests/test_gpu_rgb_train.py)
    taps = FusedRenderer(nets["gpu"]).render(ro.to(cuda), rd.to(cuda), taps=True)
    bins = [taps["bins1"].cpu().contiguous(), taps["bins2"].cpu().contiguous()]
    with oracle_encoders(), injected_bins(bins):
        out = nets["cpu"].run_torch(ro, rd, return_feats=1)
        pred = out["samvit"].reshape(1, 64, 64, 256).permute(0, 3, 1, 2).contiguous()
        pred = F.interpolate(pred, gt.shape[2:], mode="bilinear")
        lc = F.mse_loss(pred, gt, reduction="none").mean()
        lc.backward()
    assert abs(float(lg.detach()) - float(lc.detach())) <= 1e-4 * abs(float(lc.detach())), (float(lg.detach()), float(lc.detach()))
    errs = {}
    for (k, pg), (_, pc) in zip(nets["gpu"].named_parameters(), nets["cpu"].named_parameters()):
        if not pc.requires_grad:
            assert pg.grad is None, k
            continue
        a, b = pg.grad.cpu(), pc.grad
        errs[k] = float((a - b).norm() / b.norm().clamp_min(1e-12))
    print("cfg5 gradient relative errors", errs)
    assert len(errs) == 13 and max(errs.values()) < 1e-4, errs


def test_sgrid_backward_box_matches_per_corner(hip_lib, cuda, monkeypatch, diag):
    """The s_grid scatter's LDS-box aggregation (SAMNERF_SGRID_BWD=box; per
    wave and sample: corner sums in LDS, non-zero cells compacted, one atomic
    per distinct row) and the along-ray merge (SAMNERF_SGRID_BWD=run: a lane
    keeps the previous sample's corner rows pending) against the default
    per-corner form on the full-size table, a
    64x64 view and a ray set with scattered rays (boxes too big -> per-corner
    path inside the same launch): equal up to float-atomic order."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, ROW
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=9, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(14))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    perm = torch.randperm(4096, generator=torch.Generator().manual_seed(1)).to(cuda)
    ro = torch.cat([ro, ro[perm[:1000]]]).contiguous()
    rd = torch.cat([rd, rd[perm[:1000]]]).contiguous()
    N = ro.shape[0]
    fr = FusedRenderer(net)
    rows = torch.empty(N, ROW, device=cuda)
    out = fr.render(ro, rd, rows=rows, keep_workspace=True, feats=False, own_workspace=True)
    ws = out["_workspace"]
    g = torch.randn(N, ROW, device=cuda, generator=torch.Generator(device=cuda).manual_seed(2))
    grads = {}
    for mode in ("box", "corner", "run"):
        monkeypatch.setenv("SAMNERF_SGRID_BWD", mode)
        ge = torch.zeros_like(net.s_grid.embeddings)
        fr.sgrid_backward(g, ws, ge)
        grads[mode] = ge
    b = grads["corner"]
    for mode in ("box", "run"):
        a = grads[mode]
        assert (a != 0).sum() > 10000
        # another association of the same float sums (LDS first / along the
        # ray first, then one atomic per row): relative to the tensor, not per
        # element (rows whose contributions cancel carry no relative precision
        # in any form)
        rel = ((a - b).norm() / b.norm()).item()
        mx = ((a - b).abs().max() / b.abs().max()).item()
        print(mode, "vs per-corner scatter:", rel, mx)
        assert rel < 1e-5 and mx < 1e-5, (mode, rel, mx)


def test_sgrid_backward_deterministic_mode(hip_lib, cuda):
    """the deterministic s_grid scatter (samnerf_sgrid_backward_det:
    64-bit fixed-point integer atomics, associative) gives the same bits on
    every call, and the fp32-atomic scatter's values to 1e-5 of the tensor
    (norm and max), on the full-size table with a 64x64 view plus 1000
    scattered rays; its accumulator is left zero."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, ROW
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=9, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(14))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    perm = torch.randperm(4096, generator=torch.Generator().manual_seed(1)).to(cuda)
    ro = torch.cat([ro, ro[perm[:1000]]]).contiguous()
    rd = torch.cat([rd, rd[perm[:1000]]]).contiguous()
    N = ro.shape[0]
    fr = FusedRenderer(net, deterministic=True)
    rows = torch.empty(N, ROW, device=cuda)
    ws = fr.render(ro, rd, rows=rows, keep_workspace=True, feats=False, own_workspace=True)["_workspace"]
    g = torch.randn(N, ROW, device=cuda, generator=torch.Generator(device=cuda).manual_seed(2))
    dets = []
    for _ in range(3):
        ge = torch.zeros_like(net.s_grid.embeddings)
        fr.sgrid_backward(g, ws, ge)
        dets.append(ge)
    n = net.s_grid.embeddings.numel() * 8
    (acc,) = fr._accum.values()                             # one stream: one accumulator
    assert not acc[:n].any()                                # left zero for the next call
    fr.deterministic = False
    ref = torch.zeros_like(net.s_grid.embeddings)
    fr.sgrid_backward(g, ws, ref)
    for d in dets[1:]:
        assert torch.equal(d, dets[0])
    rel = ((dets[0] - ref).norm() / ref.norm()).item()
    mx = ((dets[0] - ref).abs().max() / ref.abs().max()).item()
    print("deterministic vs fp32-atomic scatter:", rel, mx, int((ref != 0).sum()))
    # the fp32 atomics round every add in whatever order the waves reach a
    # row; the fixed-point totals are exact sums rounded once: they differ
    # at the atomic form's own order noise (measured 6.9e-7 / 1.6e-6)
    assert (ref != 0).sum() > 10000 and rel < 1e-5 and mx < 1e-5, (rel, mx)


def test_sgrid_backward_deterministic_nonfinite_and_size(hip_lib, cuda):
    """a NaN (or Inf) in grad_fsam has no fixed-point scale; the
    deterministic scatter then adds with the fp32 atomics, so the NaN / Inf
    reaches the rows its ray touches (as the reference's atomics,
    gridencoder.cu:252-349) and every other row keeps the fp32-atomic value,
    instead of turning into large finite garbage.  A finite call after it is
    bit-identical to one before it (the accumulator stays clean), and a C
    caller's accumulator smaller than samnerf_sgrid_accum_size gets
    SAMNERF_EWORKSPACE, not an out-of-bounds write."""
    import ctypes
    from samnerf_amd import ops
    from samnerf_amd._lib import lib
    from samnerf_amd.fused import FusedRenderer, ROW
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    net = make_net(spec, synth.make_params(spec, seed=5, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(32, 32, rot=synth.random_rotation(3))
    ro, rd = ops.get_rays(pose, intr, 32, 32, device=cuda)
    N = ro.shape[0]
    fr = FusedRenderer(net, deterministic=True)
    rows = torch.empty(N, ROW, device=cuda)
    ws = fr.render(ro, rd, rows=rows, keep_workspace=True, feats=False, own_workspace=True)["_workspace"]
    g = torch.randn(N, ROW, device=cuda, generator=torch.Generator(device=cuda).manual_seed(4))
    clean = torch.zeros_like(net.s_grid.embeddings)
    fr.sgrid_backward(g, ws, clean)
    for bad in (float("nan"), float("inf")):
        gb = g.clone()
        gb[17, 3] = bad                                      # ray 17, level 0, channel 3
        ge = torch.zeros_like(net.s_grid.embeddings)
        fr.sgrid_backward(gb, ws, ge)
        torch.cuda.synchronize()
        hit = ~torch.isfinite(ge)
        assert hit.any(), bad                                # propagated, as the reference's atomics
        if bad != bad:
            assert bool(torch.isnan(ge[hit]).all())
        else:                                                # +-inf, or NaN where inf met 0 / -inf
            assert bool(torch.isinf(ge[hit]).any())
        # only level 0's channel 3 rows can carry it (the bad entry's column)
        lv0 = int(net.s_grid.offsets[1])
        assert not hit[lv0:].any() and not hit[:, [0, 1, 2, 4, 5, 6, 7]].any()
        ok = ~hit
        # elsewhere the fp32-atomic sums: within their order noise of the fixed point
        assert ((ge[ok] - clean[ok]).abs().max() / clean.abs().max()).item() < 1e-5
    again = torch.zeros_like(net.s_grid.embeddings)
    fr.sgrid_backward(g, ws, again)
    assert torch.equal(again, clean)                         # the accumulator was left clean
    # C ABI: a too-small accumulator is refused before any launch
    wsb, need, m, vw = ws
    m.view_width = vw
    size = lib().samnerf_sgrid_accum_size(ctypes.byref(m))
    small = torch.zeros(size - 8, dtype=torch.uint8, device=cuda)
    rc = lib().samnerf_sgrid_backward_det(ctypes.byref(m), ctypes.c_void_p(g.data_ptr()), N,
                                          ctypes.c_void_p(again.data_ptr()), ctypes.c_void_p(small.data_ptr()),
                                          small.numel(), ctypes.c_void_p(wsb.data_ptr()), need, None)
    assert rc != 0 and b"accumulator" in lib().samnerf_last_error()


def test_distillation_steps_repeat_bit_for_bit(hip_lib, cuda):
    """Two identical config-5 steps (fused render, HIP head forward /
    backward, deterministic s_grid scatter) give identical gradients, bit
    for bit, for all 13 trained tensors: the head's dW sums its 256-ray
    chunks in a fixed order (k_ht_dw + k_ht_dw_sum) and the s_grid scatter
    runs in the deterministic mode."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    from samnerf_amd.train import sam_train_step
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=7, emb_scale=0.5, ln_jitter=0.1), cuda)
    net.train()
    for k, p in net.named_parameters():
        p.requires_grad = k.startswith("s_grid") or k.startswith("samvit_mlp")
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(10))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    gt = torch.randn(1, 256, 64, 64, device=cuda, generator=torch.Generator(device=cuda).manual_seed(1))
    fr = FusedRenderer(net, deterministic=True)
    grads = []
    for _ in range(2):
        net.zero_grad(set_to_none=True)
        _, loss = sam_train_step(fr, ro, rd, 64, 64, gt)
        loss.backward()
        grads.append({k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None})
    assert len(grads[0]) == 13
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


@pytest.mark.parametrize("n", [4096, 1000, 37])
def test_head_train_kernels_match_torch_autograd(hip_lib, cuda, n):
    """sam_head_train.hip (forward with saved activations, LayerNorm and
    leaky_relu backward, dX chain, dW over all rays) against torch autograd of
    net.samvit_mlp on the same rows, fp32: outputs and every gradient (the rows
    and the 12 head tensors) to summation-order rounding; ragged ray counts
    (partial workgroups, padded ray chunks)."""
    from samnerf_amd.fused import FusedRenderer, _SamHeadTrain, _head_params
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=11, prop_log2=10)
    net = make_net(spec, synth.make_params(spec, seed=15, emb_scale=0.5, ln_jitter=0.3), cuda)
    g = torch.Generator(device="cpu").manual_seed(5)
    rows = (torch.randn(n, 164, generator=g) * torch.rand(1, 164, generator=g) * 3).to(cuda)
    rows[:, 163] = 0.0
    G = torch.randn(n, 256, generator=g).to(cuda)
    params = _head_params(net)
    r1 = rows.clone().requires_grad_(True)
    out1 = _SamHeadTrain.apply(r1, FusedRenderer(net), *params)
    (out1 * G).sum().backward()
    g1 = [p.grad.clone() for p in params]
    for p in params:
        p.grad = None
    # the backward overwrites its (torch.empty) gradient buffers: a second
    # pass, whose buffers come back from the allocator holding the first
    # pass's values, gives the same gradients, not their double
    r1b = rows.clone().requires_grad_(True)
    (_SamHeadTrain.apply(r1b, FusedRenderer(net), *params) * G).sum().backward()
    for p, a in zip(params, g1):
        assert ((p.grad - a).norm() / a.norm().clamp_min(1e-12)).item() < 1e-5
        p.grad = None
    assert ((r1b.grad - r1.grad).norm() / r1.grad.norm()).item() < 1e-5
    r2 = rows.clone().requires_grad_(True)
    out2 = net.samvit_mlp(r2[:, :163])
    (out2 * G).sum().backward()
    g2 = [p.grad.clone() for p in params]
    assert (out1 - out2).abs().max().item() < 2e-5
    gr1, gr2 = r1.grad[:, :163], r2.grad[:, :163]
    assert ((gr1 - gr2).norm() / gr2.norm()).item() < 1e-5
    assert r1.grad[:, 163].abs().max().item() == 0.0
    names = [f"net.{i}.weight" for i in range(5)] + [f"net.{i}.bias" for i in range(5)] + ["ln.w", "ln.b"]
    errs = {nm: ((a - b).norm() / b.norm().clamp_min(1e-12)).item() for nm, a, b in zip(names, g1, g2)}
    print("head train grads", n, errs)
    assert max(errs.values()) < 1e-5, errs


def test_distillation_steps_reduce_loss(hip_lib, cuda):
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, render_sam_train
    net = _frozen_net(cuda, seed=6)
    net.train()
    pose, intr = synth.gui_camera(64, 64)
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    gen = torch.Generator(device=cuda).manual_seed(1)
    gt = torch.randn(1, 256, 64, 64, device=cuda, generator=gen)
    opt = torch.optim.Adam([p for p in net.parameters() if p.requires_grad], lr=1e-2, eps=1e-15)
    r = FusedRenderer(net)
    losses = []
    for _ in range(6):
        opt.zero_grad()
        pred = render_sam_train(r, ro, rd)["samvit"].reshape(1, 64, 64, 256).permute(0, 3, 1, 2)
        pred = F.interpolate(pred, gt.shape[2:], mode="bilinear")
        loss = F.mse_loss(pred, gt)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0], losses


def _rgb_pair(cuda, seed=12):
    """The GPU net renders through the torch path (fused = False: run_torch +
    autograd + the drop-in encoder kernels) -- what these tests pin; the HIP
    training kernels are tests/test_gpu_rgb_train.py's."""
    spec = synth.ModelSpec(with_sam=False, grid_log2=12, s_grid_log2=10, prop_log2=10)
    params = synth.make_params(spec, seed=seed, emb_scale=0.5)
    gpu = make_net(spec, params, cuda).train()
    gpu.fused = False
    return gpu, make_net(spec, params, "cpu").train()


def test_rgb_train_step_gradients_match_cpu_twin(hip_lib, cuda):
    """one RGB training step (utils.py:897-937: MSE + proposal
    + distortion losses) on the GPU -- torch ops + HIP drop-in encoder
    forward/backward kernels -- against the same graph on the CPU with the C
    oracle's encoders (tests/oracle_backend.py).  perturb=False and the twin
    at the GPU run's resampled bins, so both see the same samples; per-tensor
    relative gradient error < 3e-4 (float atomics, reassociated sums)."""
    from oracle import renderer as orc
    from oracle_backend import injected_bins, oracle_encoders, recorded_bins
    from samnerf_amd.train import rgb_train_step
    gpu, cpu = _rgb_pair(cuda)
    pose, intr = synth.gui_camera(16, 16, rot=synth.random_rotation(6))
    ro, rd = orc.get_rays(pose, intr, 16, 16)
    gt = torch.rand(256, 3, generator=torch.Generator().manual_seed(2))
    # the hash grid's input and upstream gradient on the GPU (its one call,
    # the final stage), to check the drop-in backward kernel in isolation
    seen = {}

    def grab(mod, args, out):
        seen["x"] = args[0].detach()
        out.register_hook(lambda g: seen.__setitem__("g", g.detach()))
    h = gpu.grid.register_forward_hook(grab)
    bins = []
    with recorded_bins(bins):
        _, lg, _ = rgb_train_step(gpu, ro.to(cuda), rd.to(cuda), gt.to(cuda), global_step=1, perturb=False)
    lg.backward()
    h.remove()
    # the twin samples at the GPU run's bins (an ulp of a final sample position
    # moves the fine grid levels' gradients by ~1e-2: tests/test_gpu_rgb_train.py)
    with oracle_encoders(), injected_bins([b.cpu() for b in bins]):
        _, lc, _ = rgb_train_step(cpu, ro, rd, gt, global_step=1, perturb=False)
        lc.backward()
        # (1) the kernel: oracle backward on the GPU's own (x, upstream grad)
        emb = cpu.grid.embeddings
        emb.grad = None
        cpu.grid(seen["x"].cpu(), bound=cpu.bound).backward(seen["g"].cpu())
        k_ref = emb.grad.clone()
    k_err = (gpu.grid.embeddings.grad.cpu() - k_ref).norm() / k_ref.norm()
    assert k_err < 1e-4, float(k_err)
    # (2) end to end: forward loss to fp32 rounding
    assert abs(float(lg.detach()) - float(lc.detach())) <= 1e-4 * abs(float(lc.detach())) + 1e-7, (float(lg.detach()), float(lc.detach()))
    # (3) end to end gradients at the same samples: every tensor within 3e-4
    # relative (float atomics, reassociated sums; the proposal loss's fp32
    # sums ~1e-4)
    errs = {}
    for (k, pg), (_, pc) in zip(gpu.named_parameters(), cpu.named_parameters()):
        if pc.grad is None:
            assert pg.grad is None or pg.grad.abs().sum() == 0, k
            continue
        errs[k] = float((pg.grad.cpu() - pc.grad).norm() / pc.grad.norm().clamp_min(1e-12))
    print("relative gradient errors:", {k: f"{v:.1e}" for k, v in errs.items()})
    assert all(v < 3e-4 for v in errs.values()), errs


def test_rgb_training_reduces_loss(hip_lib, cuda):
    from oracle import renderer as orc
    from samnerf_amd.train import rgb_train_step
    gpu, _ = _rgb_pair(cuda, seed=13)
    opt = torch.optim.Adam(gpu.get_params(1e-2), eps=1e-15)       # main.py:296
    pose, intr = synth.gui_camera(16, 16, rot=synth.random_rotation(7))
    ro, rd = [t.to(cuda) for t in orc.get_rays(pose, intr, 16, 16)]
    gt = torch.full((256, 3), 0.25, device=cuda)
    losses = []
    for step in range(1, 9):
        _, loss, _ = rgb_train_step(gpu, ro, rd, gt, global_step=step)     # perturbed sampling
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert losses[-1] < 0.5 * losses[0], losses


@pytest.mark.parametrize("wd", [0.0, 1e-3])
def test_fused_adam_matches_torch_adam(hip_lib, cuda, wd):
    """samnerf_adam_step (one pass, all tensors in one launch) against
    torch.optim.Adam on the same parameters and gradients over several steps:
    tensors of 16-B-vector and scalar shapes, a parameter without a gradient,
    two parameter groups."""
    from samnerf_amd.optim import FusedAdam
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(5258512 // 64, 8), (256,), (7,), (3, 163), (1,)]
    init = [torch.randn(*sh, generator=g) for sh in shapes]
    ours = [torch.nn.Parameter(x.clone().to(cuda)) for x in init]
    ref = [torch.nn.Parameter(x.clone().to(cuda)) for x in init]
    kw = dict(lr=1e-2, eps=1e-15, weight_decay=wd)
    o1 = FusedAdam([{"params": ours[:3]}, {"params": ours[3:], "lr": 3e-3}], **kw)
    o2 = torch.optim.Adam([{"params": ref[:3]}, {"params": ref[3:], "lr": 3e-3}], **kw)
    for step in range(6):
        for j, (a, b) in enumerate(zip(ours, ref)):
            if j == 2 and step % 2 == 0:                      # no grad this step: skipped
                a.grad = b.grad = None
                continue
            gr = torch.randn(a.shape, generator=g).to(cuda) * (10.0 ** (j - 2))
            a.grad, b.grad = gr.clone(), gr.clone()
        o1.step()
        o2.step()
    # rounding-level differences (torch's kernels contract some products into
    # FMAs), measured against each tensor's scale: a running mean that
    # cancels to ~0 has no meaningful relative error
    for a, b in zip(ours, ref):
        err = ((a - b).abs() / (b.abs() + 1e-3)).max().item()
        assert err < 1e-5, err
        for k in ("exp_avg", "exp_avg_sq"):
            x, y = o1.state[a][k], o2.state[b][k]
            assert (x - y).abs().max().item() <= 1e-5 * y.abs().max().item(), k
        assert int(o1.state[a]["step"]) == int(o2.state[b]["step"])



def test_distillation_step_with_ray_tiles(hip_lib, cuda):
    """render_sam_train over a 64 x 64 feature view with view_width = 64 (8 x 4
    ray tiles; the s_grid scatter reads the forward's slot-ordered samples and
    the ray-ordered row gradients): the same samvit bits and the same
    gradients (to float-atomic order) as row-major waves."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, render_sam_train
    net = _frozen_net(cuda, seed=7)
    net.train()
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(2))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    g = torch.randn(4096, 256, generator=torch.Generator().manual_seed(3)).to(cuda)
    params = [p for p in net.parameters() if p.requires_grad]
    res = []
    for vw in (0, 64):
        for p in params:
            p.grad = None
        out = render_sam_train(FusedRenderer(net), ro, rd, view_width=vw)["samvit"]
        (out * g).sum().backward()
        res.append((out.detach().cpu(), [p.grad.detach().cpu().clone() for p in params]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 1e-5
