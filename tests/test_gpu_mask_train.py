"""The --with_mask training step's instance head on the HIP kernels
(csrc/mask_head_train.hip; nerf/utils.py:941-977 under renderer.py:392-395,
:451-452).

Checked against the CPU twin -- the reference's op sequence (run_torch) with
autograd on the CPU and the C oracle's encoders (tests/oracle_backend.py),
evaluated at the HIP path's own resampled bins (oracle_backend.injected_bins,
see tests/test_gpu_rgb_train.py): the softmax / clamp / NLL loss and the
gradients of m_grid.embeddings and the three mask_mlp weights (the only
tensors the reference's loss reaches: weights and geo_feat are detached).
"""
import pytest
import torch

from helpers import make_net
from oracle import synth

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-4          # relative, per tensor: fp32 sums in another order, float atomics


def _mask_nets(cuda, n_inst=5, redundant=0, sum_after=False, seed=21, head_mode=1):
    spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="default", n_inst=n_inst,
                           redundant_instance=redundant, sum_after_mlp=sum_after, grid_log2=12,
                           prop_log2=10, m_grid_log2=12)
    params = synth.make_params(spec, seed=seed, emb_scale=0.5)
    gpu = make_net(spec, params, cuda).train()
    cpu = make_net(spec, params, "cpu").train()
    cpu.fused = False
    for n in (gpu, cpu):                     # main.py:255-262: only the mask head trains
        for k, p in n.named_parameters():
            p.requires_grad = k.startswith("m_grid") or k.startswith("mask_mlp")
    # 1: geo_feat from exact fp32 grid_mlp GEMMs and the head's training
    # forward exact fp32; 0 (the default): both f16x3 (fp32-equivalent)
    gpu.head_mode = head_mode
    return gpu, cpu


def _rays(n_side, rot):
    from oracle import renderer as orc
    pose, intr = synth.gui_camera(n_side, n_side, rot=synth.random_rotation(rot))
    return orc.get_rays(pose, intr, n_side, n_side)


def _fused_bins(net, ro, rd):
    from samnerf_amd.fused import FusedRenderer
    out = FusedRenderer(net).render(ro, rd, taps=True)
    return [out["bins1"].contiguous().cpu(), out["bins2"].contiguous().cpu()]


def _grad_errors(gpu, cpu):
    errs = {}
    for (k, pa), (_, pb) in zip(gpu.named_parameters(), cpu.named_parameters()):
        if pb.grad is None:
            assert pa.grad is None, k
            continue
        a, b = pa.grad.detach().cpu(), pb.grad.detach()
        errs[k] = float((a - b).norm() / b.norm().clamp_min(1e-12))
    return errs


@pytest.mark.parametrize("n_inst,redundant,sum_after,head_mode",
                         [(5, 0, False, 1), (2, 0, True, 1), (32, 0, False, 1), (1, 0, False, 1),
                          (5, 0, False, 0), (32, 0, False, 0), (2, 0, True, 0)])
def test_fused_mask_step_matches_cpu_twin(hip_lib, cuda, n_inst, redundant, sum_after, head_mode):
    """head_mode 1: the exact fp32 training forward (k_mt_fwd); 0 (the
    default): the f16x3 forward (k_mt_fwd16); the backward is exact fp32 in
    both."""
    from oracle_backend import injected_bins, oracle_encoders
    from samnerf_amd.train import mask_train_step
    gpu, cpu = _mask_nets(cuda, n_inst, redundant, sum_after, head_mode=head_mode)
    ro, rd = _rays(16, 4)
    gt = torch.randint(0, n_inst, (256,), generator=torch.Generator().manual_seed(3))
    bins = _fused_bins(gpu, ro.to(cuda), rd.to(cuda))
    pred, loss = mask_train_step(gpu, ro.to(cuda), rd.to(cuda), gt.to(cuda))
    loss.backward()
    with oracle_encoders(), injected_bins(bins):
        pred_c, loss_c = mask_train_step(cpu, ro, rd, gt)
        loss_c.backward()
    assert abs(float(loss.detach()) - float(loss_c.detach())) <= 1e-5 * abs(float(loss_c.detach())) + 1e-7, (float(loss.detach()), float(loss_c.detach()))
    errs = _grad_errors(gpu, cpu)
    print("relative gradient errors:", {k: f"{v:.1e}" for k, v in errs.items()})
    assert set(errs) == {"m_grid.embeddings", "mask_mlp.0.net.0.weight", "mask_mlp.0.net.1.weight",
                         "mask_mlp.0.net.2.weight"}, errs
    bad = {k: v for k, v in errs.items() if v > GRAD_TOL}
    assert not bad, bad


@pytest.mark.parametrize("head_mode", [1, 0])
def test_fused_mask_logits_match_inference_head(hip_lib, cuda, head_mode):
    """The training forward's logits (k_mt_fwd / k_mt_fwd16 + k_mt_logits) equal
    the inference head's (k_mask_head) in the same head_mode to fp32 level."""
    from samnerf_amd.fused import FusedRenderer, render_mask_train
    gpu, _ = _mask_nets(cuda, n_inst=7, head_mode=head_mode)
    ro, rd = _rays(24, 5)
    ro, rd = ro.to(cuda), rd.to(cuda)
    fr = FusedRenderer(gpu)
    with torch.enable_grad():
        out = render_mask_train(fr, ro, rd)
    with torch.no_grad():
        ref = fr.render(ro, rd, mask=True, feats=False)
    lt, li = out["instance_mask_logits"].detach(), ref["instance_mask_logits"]
    assert (lt - li).abs().max().item() <= 1e-5 * li.abs().max().item() + 1e-7
    for k in ("image", "depth", "weights_sum"):
        assert torch.equal(out[k], ref[k]), k


def test_train_mode_mask_render_runs_the_training_kernels(hip_lib, cuda, monkeypatch):
    """NeRFRenderer.run in train mode under grad with return_mask=1 takes the
    HIP mask-training path (never run_torch) and returns logits with grad."""
    gpu, _ = _mask_nets(cuda)
    ro, rd = _rays(8, 2)

    def boom(*a, **k):
        raise AssertionError("run_torch called")
    monkeypatch.setattr(type(gpu), "run_torch", boom)
    out = gpu.render(ro.to(cuda), rd.to(cuda), staged=False, bg_color=1, perturb=False,
                     update_proposal=False, return_feats=0, return_mask=1)
    assert out["instance_mask_logits"].requires_grad
    assert out["instance_mask_logits"].grad_fn is not None


def test_fused_mask_step_repeatable(hip_lib, cuda):
    """Two identical steps: the same loss and weight gradients to float-atomic
    reassociation (the m_grid scatter and dW are float atomics, as the
    reference's encoder backward)."""
    from samnerf_amd.train import mask_train_step
    gpu, _ = _mask_nets(cuda)
    ro, rd = _rays(16, 7)
    gt = torch.randint(0, 5, (256,), generator=torch.Generator().manual_seed(4)).to(cuda)
    grads = []
    for _ in range(2):
        gpu.zero_grad(set_to_none=True)
        _, loss = mask_train_step(gpu, ro.to(cuda), rd.to(cuda), gt)
        loss.backward()
        grads.append({k: p.grad.clone() for k, p in gpu.named_parameters() if p.grad is not None})
    for k in grads[0]:
        a, b = grads[0][k], grads[1][k]
        assert float((a - b).norm()) <= 1e-6 * float(b.norm()) + 1e-12, k


# ------------------------------------------------------------- adaptive heads
def _adaptive_nets(cuda, adaptive_type, n_inst, seed=22):
    spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="adaptive", adaptive_type=adaptive_type,
                           n_inst=n_inst, sum_after_mlp=True, grid_log2=12, prop_log2=10)
    params = synth.make_params(spec, seed=seed, emb_scale=0.5)
    gpu = make_net(spec, params, cuda).train()
    cpu = make_net(spec, params, "cpu").train()
    cpu.fused = False
    for n in (gpu, cpu):                     # main.py:255-262: only the mask head trains
        for k, p in n.named_parameters():
            p.requires_grad = k.startswith("mask_mlp")
    gpu.head_mode = 1                        # grid_mlp intermediates from exact fp32 GEMMs
    return gpu, cpu


@pytest.mark.parametrize("adaptive_type,n_inst", [("density", 5), ("density", 32), ("rgb", 3)])
def test_fused_adaptive_mask_step_matches_cpu_twin(hip_lib, cuda, adaptive_type, n_inst):
    """--mask_mlp_type adaptive --adaptive_mlp_type density --sum_after_mlp, the
    reference's own scripts/train_mask.sh:16,20,21 (and the 'rgb' variant):
    loss and the gradient of every mask_mlp Linear against the CPU twin (the
    reference's per-sample chain + weighted sum with autograd) at the HIP
    path's own bins.  The fused path applies the chain to each ray's weighted
    input sums (the head is linear): rounding-level reassociation."""
    from oracle_backend import injected_bins, oracle_encoders
    from samnerf_amd.train import mask_train_step
    gpu, cpu = _adaptive_nets(cuda, adaptive_type, n_inst)
    ro, rd = _rays(16, 6)
    gt = torch.randint(0, n_inst, (256,), generator=torch.Generator().manual_seed(5))
    bins = _fused_bins(gpu, ro.to(cuda), rd.to(cuda))
    pred, loss = mask_train_step(gpu, ro.to(cuda), rd.to(cuda), gt.to(cuda))
    loss.backward()
    with oracle_encoders(), injected_bins(bins):
        pred_c, loss_c = mask_train_step(cpu, ro, rd, gt)
        loss_c.backward()
    assert abs(float(loss.detach()) - float(loss_c.detach())) <= 1e-5 * abs(float(loss_c.detach())) + 1e-7, (float(loss.detach()), float(loss_c.detach()))
    errs = _grad_errors(gpu, cpu)
    print(adaptive_type, "relative gradient errors:", {k: f"{v:.1e}" for k, v in errs.items()})
    n_layers = 6 if adaptive_type == "density" else 8
    assert set(errs) == {f"mask_mlp.{i}.weight" for i in range(n_layers)}, errs
    bad = {k: v for k, v in errs.items() if v > GRAD_TOL}
    assert not bad, bad


def test_train_mode_adaptive_render_runs_the_training_kernels(hip_lib, cuda, monkeypatch):
    """NeRFRenderer.run in train mode under grad with return_mask=1 for the
    train_mask.sh head takes the HIP path (never run_torch); the training
    logits equal the inference head's (k_final<AD> + k_mask_eff: E . X) to
    rounding; two identical steps give bitwise-identical weight gradients
    (fixed-order sums, no atomics)."""
    from samnerf_amd.fused import FusedRenderer
    gpu, _ = _adaptive_nets(cuda, "density", 4)
    ro, rd = _rays(12, 3)
    ro, rd = ro.to(cuda), rd.to(cuda)

    def boom(*a, **k):
        raise AssertionError("run_torch called")
    monkeypatch.setattr(type(gpu), "run_torch", boom)
    grads = []
    for _ in range(2):
        gpu.zero_grad(set_to_none=True)
        out = gpu.render(ro, rd, staged=False, bg_color=1, perturb=False, update_proposal=False,
                         return_feats=0, return_mask=1)
        lg = out["instance_mask_logits"]
        assert lg.requires_grad and lg.grad_fn is not None
        (lg * torch.linspace(-1, 1, lg.numel(), device=cuda).view_as(lg)).sum().backward()
        grads.append({k: p.grad.clone() for k, p in gpu.named_parameters() if p.grad is not None})
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k
    with torch.no_grad():
        ref = FusedRenderer(gpu).render(ro, rd, mask=True, feats=False)["instance_mask_logits"]
    err = (lg.detach() - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item() + 1e-7, err
