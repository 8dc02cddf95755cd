"""The RGB training step on the HIP training kernels (samnerf_rgb_train_step,
csrc/rgb_train.hip; SURVEY.md 8f-2, nerf/utils.py:897-937).

Checked against:
  * the CPU twin -- the reference's op sequence (run_torch) with autograd on
    the CPU and the C oracle's encoders (tests/oracle_backend.py), perturb off;
  * the torch path on the GPU (run_torch + autograd with the drop-in encoder
    kernels) with perturb on, both drawing the same perturbed positions;
  * a float64 twin of the step (oracle_backend.float64_twin).
Every comparison evaluates the reference at the HIP path's own resampled bins
(oracle_backend.injected_bins, the bins read through the render's parity
taps; they agree with the reference's own to ~1e-7): the proposal MLPs sum in
another order than torch's GEMMs, the bins then differ by an ulp, and an ulp
of a final sample position moves the grid / grid_mlp gradients by ~1e-2
(fine levels resolve 2^-12 of the range) -- a real difference of the sampled
function, not arithmetic error.  At the same bins: every gradient within
GRAD_TOL of the reference (float atomics, reassociated sums), and within 2x
of the fp32 CPU twin's own distance to the float64 twin.
"""
import contextlib

import pytest
import torch
import torch.nn.functional as F

from helpers import make_net
from oracle import synth

pytestmark = pytest.mark.gpu


def _rgb_nets(cuda, seed=12, log2=(12, 10), devices=("cuda", "cpu")):
    """Identical networks; every one after the first renders through the torch
    path (fused = False: run_torch + autograd with the drop-in encoder kernels),
    the reference's op sequence the fused step is checked against."""
    spec = synth.ModelSpec(with_sam=False, grid_log2=log2[0], s_grid_log2=10, prop_log2=log2[1])
    params = synth.make_params(spec, seed=seed, emb_scale=0.5)
    nets = [make_net(spec, params, cuda if d == "cuda" else "cpu").train() for d in devices]
    for n in nets[1:]:
        n.fused = False
    return nets


def _rays(n_side, rot, cuda=None):
    from oracle import renderer as orc
    pose, intr = synth.gui_camera(n_side, n_side, rot=synth.random_rotation(rot))
    ro, rd = orc.get_rays(pose, intr, n_side, n_side)
    if cuda is not None:
        ro, rd = ro.to(cuda), rd.to(cuda)
    return ro, rd


GRAD_TOL = 3e-4          # relative, per tensor (the proposal loss's fp32 sums: ~1e-4 each side)


def _compare_grads(net_a, net_b, tol=GRAD_TOL):
    worst = {}
    for (k, pa), (_, pb) in zip(net_a.named_parameters(), net_b.named_parameters()):
        if pb.grad is None:
            assert pa.grad is None, k
            continue
        a, b = pa.grad.detach().cpu(), pb.grad.detach().cpu()
        worst[k] = float((a - b).norm() / b.norm().clamp_min(1e-12))
    print("relative gradient errors:", {k: f"{v:.1e}" for k, v in worst.items()})
    bad = {k: v for k, v in worst.items() if v > tol}
    assert not bad, bad
    return worst


def _fused_bins(net, ro, rd, cnf=None, pert=None):
    """The HIP proposal kernels' resampled bins for these rays ([N, 65],
    [N, 33]; the training step runs the same kernels, proposal_forward), read
    through the render's parity taps."""
    from samnerf_amd.fused import FusedRenderer
    out = FusedRenderer(net).render(ro, rd, cam_near_far=cnf, taps=True, perturb=pert or False)
    return [out["bins1"].contiguous(), out["bins2"].contiguous()]


def _draws(seed, n, device):
    """perturb=True's draws (fused.perturbed_positions) from a seeded generator."""
    from samnerf_amd.fused import perturbed_positions
    torch.manual_seed(seed)
    return perturbed_positions(n, [128, 64, 32], device)


def test_fused_rgb_step_matches_cpu_twin(hip_lib, cuda):
    """perturb=False, update_proposal on (step 1): image, the four loss terms
    and all 11 gradients against autograd of the reference's op sequence on
    the CPU with the oracle encoders."""
    from oracle_backend import oracle_encoders
    from samnerf_amd.train import rgb_train_step, rgb_train_step_fused
    from oracle_backend import injected_bins
    gpu, cpu = _rgb_nets(cuda)
    ro, rd = _rays(16, 6)
    gt = torch.rand(256, 3, generator=torch.Generator().manual_seed(2))
    bins = [b.cpu() for b in _fused_bins(gpu, ro.to(cuda), rd.to(cuda))]
    img, loss, out = rgb_train_step_fused(gpu, ro.to(cuda), rd.to(cuda), gt.to(cuda), global_step=1,
                                          perturb=False)
    with oracle_encoders(), injected_bins(bins):
        img_c, loss_c, out_c = rgb_train_step(cpu, ro, rd, gt, global_step=1, perturb=False)
        loss_c.backward()
    assert (img.cpu() - img_c.detach()).abs().max().item() < 1e-5
    assert (out["weights_sum"].cpu() - out_c["weights_sum"].detach()).abs().max().item() < 1e-5
    for k in ("proposal_loss", "distort_loss"):
        a, b = (float(torch.as_tensor(x).detach()) for x in (out[k], out_c[k]))
        assert abs(a - b) <= 1e-4 * abs(b) + 1e-8, (k, a, b)
    assert abs(float(loss.detach()) - float(loss_c.detach())) <= 1e-4 * abs(float(loss_c.detach())) + 1e-7
    _compare_grads(gpu, cpu)


def _float64_twin_errors(nets_fp32, cpu, ro, rd, gt, global_step=1, bins=None):
    """Relative gradient errors of each fp32 network against a float64 twin
    of the step (tests/oracle_backend.float64_twin: the reference's op
    sequence in float64 at the fp32 run's own sample positions), the fp32 CPU
    twin (C oracle encoders) among them.  bins: the proposal stages'
    resampled bins to evaluate the step at (injected_bins), e.g. the HIP
    path's -- the grid / grid_mlp gradients move ~1e-2 when the final sample
    positions move by one ulp (fine levels: a cell is ~2^-12 of the range),
    so the twins must sample where the kernels did."""
    import copy
    from oracle_backend import float64_twin, injected_bins, oracle_encoders
    from samnerf_amd.train import rgb_train_step
    n64 = copy.deepcopy(cpu).double()
    rec = []
    with oracle_encoders(record=rec), injected_bins(bins or []) if bins else contextlib.nullcontext():
        _, loss_c, _ = rgb_train_step(cpu, ro, rd, gt, global_step=global_step, perturb=False)
        loss_c.backward()
    with float64_twin(grid_inputs=rec), injected_bins(bins or []) if bins else contextlib.nullcontext():
        _, loss64, _ = rgb_train_step(n64, ro.double(), rd.double(), gt.double(), global_step=global_step,
                                      perturb=False)
        loss64.backward()
    errs = {}
    for name, net in list(nets_fp32.items()) + [("cpu_fp32", cpu)]:
        e = {}
        for (k, a), (_, b) in zip(net.named_parameters(), n64.named_parameters()):
            if b.grad is None:
                continue
            e[k] = ((a.grad.detach().cpu().double() - b.grad).norm() / b.grad.norm().clamp_min(1e-300)).item()
        errs[name] = e
    return errs, float(loss64.detach())


@pytest.mark.parametrize("lam", [(1.0, 0.02, 0.0), (1.0, 0.0, 0.0), (0.0, 0.0, 0.0), (1.0, 0.02, 1e-3)],
                         ids=["default", "no_distort", "mse_only", "entropy"])
def test_fused_rgb_step_vs_float64_twin(hip_lib, cuda, lam):
    """Every gradient of the HIP training step, the density path's grid /
    grid_mlp tensors included, is as close to the float64 twin of the step as
    the fp32 CPU twin is (within 2x, or 1e-5 relative), at the reference's
    table sizes' small stand-in (grid 2^12, proposal 2^10), perturb off; with
    the default loss weights (lambda_proposal 1, lambda_distort 0.02), without
    the distortion term, MSE alone, and with the entropy term."""
    from samnerf_amd.fused import FusedRenderer
    from samnerf_amd.train import rgb_train_step_fused
    gpu, cpu = _rgb_nets(cuda)
    for n in (gpu, cpu):
        n.opt.lambda_proposal, n.opt.lambda_distort, n.opt.lambda_entropy = lam
    ro, rd = _rays(16, 6)
    gt = torch.rand(256, 3, generator=torch.Generator().manual_seed(2))
    # the bins the HIP proposal kernels resample (the step runs the same
    # kernels, proposal_forward): read through the render's parity taps
    taps = FusedRenderer(gpu).render(ro.to(cuda), rd.to(cuda), taps=True)
    bins = [taps["bins1"].cpu().contiguous(), taps["bins2"].cpu().contiguous()]
    _, loss, _ = rgb_train_step_fused(gpu, ro.to(cuda), rd.to(cuda), gt.to(cuda), global_step=1, perturb=False)
    errs, loss64 = _float64_twin_errors({"hip": gpu}, cpu, ro, rd, gt, bins=bins)
    print("relative gradient error vs float64 twin (hip | cpu fp32):")
    for k in errs["hip"]:
        print(f"  {k:32s} {errs['hip'][k]:.2e} | {errs['cpu_fp32'][k]:.2e}")
    assert abs(float(loss.detach()) - loss64) <= 2e-6 * abs(loss64)
    bad = {k: (v, errs["cpu_fp32"][k]) for k, v in errs["hip"].items()
           if v > max(2.0 * errs["cpu_fp32"][k], 1e-5)}
    assert not bad, bad


def test_fused_rgb_step_matches_torch_path_perturbed(hip_lib, cuda):
    """perturb=True (the reference's training sampling): the fused step and the
    torch path draw the same perturbed positions from the same seed and agree
    on image, loss and gradients; 64 x 64 rays at the reference's table sizes
    (grid 2^19, proposal 2^17)."""
    from samnerf_amd.train import rgb_train_step, rgb_train_step_fused
    a, b = _rgb_nets(cuda, seed=21, log2=(19, 17), devices=("cuda", "cuda"))
    ro, rd = _rays(64, 3, cuda)
    gt = torch.rand(4096, 3, generator=torch.Generator().manual_seed(5)).to(cuda)
    from oracle_backend import injected_bins
    draws = _draws(11, 4096, cuda)
    bins = _fused_bins(a, ro, rd, pert=draws)
    img, loss, out = rgb_train_step_fused(a, ro, rd, gt, global_step=1, perturb=draws)
    torch.manual_seed(11)
    with injected_bins(bins):
        img_t, loss_t, out_t = rgb_train_step(b, ro, rd, gt, global_step=1)
        loss_t.backward()
    assert (img - img_t.detach()).abs().max().item() < 1e-5
    assert abs(float(loss.detach()) - float(loss_t.detach())) <= 1e-4 * abs(float(loss_t.detach())) + 1e-7
    assert abs(float(out["proposal_loss"]) - float(out_t["proposal_loss"])) <= \
        1e-4 * abs(float(out_t["proposal_loss"])) + 1e-8
    _compare_grads(a, b)


def test_fused_rgb_step_without_proposal_update(hip_lib, cuda):
    """utils.py:912-913: after step 3000 the proposal networks train every 5th
    step only; on the other steps their .grad stays None (no proposal loss)."""
    from samnerf_amd.train import rgb_train_step, rgb_train_step_fused
    a, b = _rgb_nets(cuda, seed=4, devices=("cuda", "cuda"))
    ro, rd = _rays(16, 2, cuda)
    gt = torch.rand(256, 3, generator=torch.Generator().manual_seed(8)).to(cuda)
    from oracle_backend import injected_bins
    draws = _draws(3, 256, cuda)
    bins = _fused_bins(a, ro, rd, pert=draws)
    _, loss, _ = rgb_train_step_fused(a, ro, rd, gt, global_step=3001, perturb=draws)
    torch.manual_seed(3)
    with injected_bins(bins):
        _, loss_t, _ = rgb_train_step(b, ro, rd, gt, global_step=3001)
        loss_t.backward()
    assert abs(float(loss.detach()) - float(loss_t.detach())) <= 1e-4 * abs(float(loss_t.detach())) + 1e-7
    assert all(p.grad is None for p in a.prop_encoders.parameters())
    assert all(p.grad is None for p in a.prop_mlp.parameters())
    _compare_grads(a, b)


def test_fused_rgb_step_entropy_and_background(hip_lib, cuda):
    """lambda_entropy > 0 (utils.py:926-929) and an RGBA target composited on the
    background (utils.py:901-906), perturb off, against the torch path."""
    from samnerf_amd.train import rgb_train_step, rgb_train_step_fused
    a, b = _rgb_nets(cuda, seed=9, devices=("cuda", "cuda"))
    for n in (a, b):
        n.opt.lambda_entropy = 1e-3
    ro, rd = _rays(16, 5, cuda)
    gt = torch.rand(256, 4, generator=torch.Generator().manual_seed(1)).to(cuda)
    from oracle_backend import injected_bins
    bins = _fused_bins(a, ro, rd)
    _, loss, out = rgb_train_step_fused(a, ro, rd, gt, global_step=2, perturb=False)
    with injected_bins(bins):
        _, loss_t, _ = rgb_train_step(b, ro, rd, gt, global_step=2, perturb=False)
        loss_t.backward()
    assert float(out["entropy"]) > 0
    assert abs(float(loss.detach()) - float(loss_t.detach())) <= 1e-4 * abs(float(loss_t.detach())) + 1e-7
    _compare_grads(a, b)


def test_fused_rgb_training_reduces_loss(hip_lib, cuda):
    """Eight fused steps with FusedAdam (main.py:296: Adam lr 1e-2, eps 1e-15):
    the loss halves, as on the torch path (test_gpu_train.py)."""
    from samnerf_amd.optim import FusedAdam
    from samnerf_amd.train import rgb_train_step_fused
    (net,) = _rgb_nets(cuda, seed=13, devices=("cuda",))
    opt = FusedAdam(net.get_params(1e-2), eps=1e-15)
    ro, rd = _rays(16, 7, cuda)
    gt = torch.full((256, 3), 0.25, device=cuda)
    losses = []
    for step in range(1, 9):
        opt.zero_grad(set_to_none=True)
        _, loss, _ = rgb_train_step_fused(net, ro, rd, gt, global_step=step)
        opt.step()
        losses.append(float(loss.detach()))
    assert losses[-1] < 0.5 * losses[0], losses


@pytest.mark.parametrize("n_rays", [1, 37, 100])
def test_fused_rgb_step_ragged_batches(hip_lib, cuda, n_rays):
    """Ray counts that fill no wave (1), part of one (37) and part of two (100
    rays = 3,200 final samples, a ragged last wave of the ray-major kernels),
    with a per-ray cam_near_far (renderer.py:234-236): against the torch path."""
    from samnerf_amd.train import rgb_train_step, rgb_train_step_fused
    a, b = _rgb_nets(cuda, seed=17, devices=("cuda", "cuda"))
    ro, rd = _rays(16, 9, cuda)
    ro, rd = ro[:n_rays].contiguous(), rd[:n_rays].contiguous()
    g = torch.Generator().manual_seed(n_rays)
    gt = torch.rand(n_rays, 3, generator=g).to(cuda)
    cnf = torch.stack([torch.full((n_rays,), 0.3), 0.8 + 2 * torch.rand(n_rays, generator=g)], -1).to(cuda)
    from oracle_backend import injected_bins
    draws = _draws(n_rays, n_rays, cuda)
    bins = _fused_bins(a, ro, rd, cnf=cnf, pert=draws)
    img, loss, _ = rgb_train_step_fused(a, ro, rd, gt, global_step=1, cam_near_far=cnf, perturb=draws)
    torch.manual_seed(n_rays)
    with injected_bins(bins):
        img_t, loss_t, _ = rgb_train_step(b, ro, rd, gt, global_step=1, cam_near_far=cnf)
        loss_t.backward()
    assert (img - img_t.detach()).abs().max().item() < 1e-5
    assert abs(float(loss.detach()) - float(loss_t.detach())) <= 1e-4 * abs(float(loss_t.detach())) + 1e-7
    _compare_grads(a, b)


def test_fused_rgb_step_deterministic_weight_gradients(hip_lib, cuda):
    """The MLP weight gradients are slab sums in a fixed order (no float
    atomics): two identical steps give identical bits; the grid gradients
    (float atomics, as the reference's backward) agree to rounding."""
    from samnerf_amd.train import rgb_train_step_fused
    (net,) = _rgb_nets(cuda, seed=19, devices=("cuda",))
    ro, rd = _rays(32, 4, cuda)
    gt = torch.rand(1024, 3, generator=torch.Generator().manual_seed(6)).to(cuda)
    res = []
    for _ in range(2):
        net.zero_grad(set_to_none=True)
        rgb_train_step_fused(net, ro, rd, gt, global_step=1, perturb=False)
        res.append({k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None})
    for k in res[0]:
        if "mlp" in k:
            assert torch.equal(res[0][k], res[1][k]), k
        else:
            err = ((res[0][k] - res[1][k]).norm() / res[1][k].norm().clamp_min(1e-30)).item()
            assert err < 1e-5, (k, err)


def test_train_mode_render_runs_the_training_kernels(hip_lib, cuda):
    """NeRFRenderer.run in train mode under grad (the reference Trainer's own
    call, utils.py:913-931 + loss.backward()) dispatches to the HIP training
    kernels through an autograd Function: the Trainer-shaped step
    (rgb_train_step: render, criterion, extra losses, backward) equals the
    one-call samnerf_rgb_train_step (float-atomic order aside) and the torch
    path."""
    from samnerf_amd.train import rgb_train_step, rgb_train_step_fused
    a, b, c = _rgb_nets(cuda, seed=23, devices=("cuda", "cuda", "cuda"))
    c.fused = True                                   # the autograd path
    ro, rd = _rays(32, 8, cuda)
    gt = torch.rand(1024, 3, generator=torch.Generator().manual_seed(9)).to(cuda)
    torch.manual_seed(5)
    _, loss_a, _ = rgb_train_step_fused(a, ro, rd, gt, global_step=1)
    from oracle_backend import injected_bins
    bins = _fused_bins(a, ro, rd, pert=_draws(5, 1024, cuda))
    torch.manual_seed(5)
    with injected_bins(bins):
        _, loss_b, _ = rgb_train_step(b, ro, rd, gt, global_step=1)
        loss_b.backward()
    torch.manual_seed(5)
    img_c, loss_c, out_c = rgb_train_step(c, ro, rd, gt, global_step=1)
    assert "proposal_loss" in out_c and "distort_loss" in out_c and out_c["num_points"] == 1024 * 32
    assert out_c["weights"].shape == (1024, 32) and out_c["weights"].requires_grad   # as renderer.py:350
    torch.testing.assert_close(out_c["weights"].sum(-1), out_c["weights_sum"].detach(), rtol=1e-5, atol=1e-6)
    assert img_c.requires_grad and loss_c.requires_grad
    loss_c.backward()
    assert abs(float(loss_c.detach()) - float(loss_a.detach())) <= 1e-6 * abs(float(loss_a.detach()))
    for (k, pa), (_, pc) in zip(a.named_parameters(), c.named_parameters()):
        err = float((pa.grad - pc.grad).norm() / pa.grad.norm().clamp_min(1e-30))
        assert err < 1e-5, (k, err)
    _compare_grads(c, b)


def test_fused_rgb_step_accumulates_into_existing_grad(hip_lib, cuda):
    """Like loss.backward(), a second fused step adds into .grad: two steps
    on the same batch leave twice the gradient of one."""
    from samnerf_amd.train import rgb_train_step_fused
    (net,) = _rgb_nets(cuda, seed=29, devices=("cuda",))
    ro, rd = _rays(16, 3, cuda)
    gt = torch.rand(256, 3, generator=torch.Generator().manual_seed(4)).to(cuda)
    rgb_train_step_fused(net, ro, rd, gt, global_step=1, perturb=False)
    one = {k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None}
    rgb_train_step_fused(net, ro, rd, gt, global_step=1, perturb=False)
    for k, p in net.named_parameters():
        if k in one:
            err = ((p.grad - 2 * one[k]).norm() / one[k].norm().clamp_min(1e-30)).item()
            assert err < 1e-5, (k, err)


def test_autograd_rgb_step_with_depth_and_weights_sum_loss(hip_lib, cuda):
    """A loss on depth.mean() + weights_sum.mean() (their gradients arrive as
    expanded, non-contiguous tensors) through the autograd Function equals the
    torch path's gradients (the converted gradients must stay alive
    through the C call)."""
    a, b = _rgb_nets(cuda, seed=31, devices=("cuda", "cuda"))
    a.fused = True
    ro, rd = _rays(16, 4, cuda)
    from oracle_backend import injected_bins
    bins = _fused_bins(a, ro, rd)
    outs = []
    for n in (a, b):
        with injected_bins(bins) if n is b else contextlib.nullcontext():
            o = n.render(ro, rd, staged=False, bg_color=1, perturb=False, update_proposal=True,
                         return_feats=0)
        loss = (o["image"].mean() + 0.3 * o["depth"].mean() + 2.0 * o["weights_sum"].mean()
                + o["proposal_loss"])
        loss.backward()
        outs.append(float(loss.detach()))
    assert abs(outs[0] - outs[1]) <= 1e-5 * abs(outs[1])
    _compare_grads(a, b)


def test_fused_render_weights_are_differentiable(hip_lib, cuda):
    """results['weights'] carries gradient on the fused training path as in the
    reference (renderer.py:350): a loss on the per-sample weights (plus depth
    and image, no proposal / distortion terms) against the torch path's
    autograd at the same bins."""
    from oracle_backend import injected_bins
    a, b = _rgb_nets(cuda, seed=14, devices=("cuda", "cuda"))
    ro, rd = _rays(16, 4, cuda)
    bins = _fused_bins(a, ro, rd)
    ramp = torch.linspace(0.0, 1.0, 32, device=cuda)

    def loss_of(net):
        out = net.render(ro, rd, staged=False, perturb=False, bg_color=1.0)
        w = out["weights"]
        assert w.requires_grad
        return (w * ramp).sum() / w.shape[0] + 1e-3 * out["depth"].mean() + out["image"].mean()

    la = loss_of(a)
    la.backward()
    with injected_bins(bins):
        lb = loss_of(b)
        lb.backward()
    assert abs(float(la.detach()) - float(lb.detach())) <= 1e-5 * abs(float(lb.detach())) + 1e-7
    _compare_grads(a, b)
