"""Perturbed sampling (run(perturb=True), nerf/renderer.py:266-271 and
sample_pdf's :100-101).

CPU: the oracle against the reference's own perturbed render
(tests/golden/render_perturbed_sam.npz, tools/make_golden.py), and the
product's draw helper (fused.perturbed_positions) against the positions the
reference drew from the same seed.

GPU: the fused path fed the golden's positions against the golden; a whole
512x512 perturbed view with the proposal stages' searchsorted indices
bit-exact against the oracle on the kernels' own weights and perturbed u;
NeRFRenderer.run(perturb=True) (fused, device generator) against run_torch
(perturb=True) from the same seed.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from helpers import make_net, oracle_for, spec_from_fixture
from oracle import renderer as orc
from oracle import synth

TOL = 1e-3


def _fixture():
    fx = np.load(os.path.join(GOLDEN, "render_perturbed_sam.npz"))
    spec = spec_from_fixture(fx)
    params = synth.make_params(spec, seed=int(fx["seed"]), emb_scale=float(fx["emb_scale"]),
                               ln_jitter=float(fx["ln_jitter"]))
    draws = tuple(torch.from_numpy(fx[k]) for k in ("bins0", "u1", "u2"))
    return fx, spec, params, draws


def test_oracle_perturbed_matches_reference_golden(oracle_lib):
    fx, spec, params, draws = _fixture()
    H, W = int(fx["H"]), int(fx["W"])
    ro, rd = torch.from_numpy(fx["rays_o"]), torch.from_numpy(fx["rays_d"])
    model = orc.OracleNeRF(spec, params)
    given = model.run(ro, rd, return_feats=1, H=H, W=W, perturbed=draws)
    torch.manual_seed(int(fx["torch_seed"]))
    drawn = model.run(ro, rd, return_feats=1, H=H, W=W, perturb=True)
    for out in (given, drawn):
        for k in ("image", "depth", "weights_sum"):
            assert np.array_equal(out[k].numpy(), fx[k]), k
        assert np.array_equal(out["samvit"].reshape(H * W, -1).numpy(), fx["samvit"])


def test_perturbed_positions_draw_like_the_reference():
    """The product's helper consumes torch's generator as the reference's run
    does (same shapes, same order, same expressions): identical positions."""
    from samnerf_amd.fused import perturbed_positions
    fx, spec, _, draws = _fixture()
    torch.manual_seed(int(fx["torch_seed"]))
    got = perturbed_positions(draws[0].shape[0], list(spec.num_steps), "cpu")
    for g, d in zip(got, draws):
        assert torch.equal(g, d)
    # u stays nondecreasing up to rounding and inside [0, 1]; bins0 is clamped
    assert (draws[0] >= 0).all() and (draws[0] <= 1).all()
    for u in draws[1:]:
        assert (u >= 0).all() and (u <= 1).all()
        assert (u[:, 1:] - u[:, :-1]).min() > -1e-6


@pytest.mark.gpu
def test_perturbed_positions_on_the_device_draw_like_the_reference(cuda):
    """On the GPU: the helper's draws equal the reference's expressions run on
    the device from the same seed -- the stage-0 bins from a device linspace
    (renderer.py:264-271), sample_pdf's u from a CPU linspace moved to the
    device (renderer.py:97), which can differ from a device linspace in the
    last bit."""
    from samnerf_amd.fused import perturbed_positions
    N, steps = 4096, [128, 64, 32]
    torch.cuda.manual_seed(11)
    got = perturbed_positions(N, steps, cuda)
    torch.cuda.manual_seed(11)
    T0 = steps[0]
    bins = torch.linspace(0, 1, T0 + 1, device=cuda).unsqueeze(0).expand(N, -1)
    want = [(bins + (torch.rand_like(bins) - 0.5) / T0).clamp(0, 1)]
    for T in (steps[1] + 1, steps[2] + 1):
        u = torch.linspace(0.5 / T, 1 - 0.5 / T, steps=T).to(cuda).expand(N, T)
        want.append(u + (torch.rand_like(u) - 0.5) / T)
    for g, w in zip(got, want):
        assert g.device.type == "cuda" and torch.equal(g, w)


@pytest.mark.gpu
@pytest.mark.parametrize("head_mode", [0, 1])
def test_fused_perturbed_matches_reference_golden(hip_lib, cuda, monkeypatch, head_mode):
    from samnerf_amd.fused import FusedRenderer
    fx, spec, params, draws = _fixture()
    net = make_net(spec, params, cuda)
    ro = torch.from_numpy(fx["rays_o"]).to(cuda)
    rd = torch.from_numpy(fx["rays_d"]).to(cuda)
    out = FusedRenderer(net, head_mode=head_mode).render(ro, rd, perturb=tuple(d.to(cuda) for d in draws))
    errs = {k: (out[k].cpu() - torch.from_numpy(fx[k])).abs().max().item()
            for k in ("image", "depth", "weights_sum", "samvit")}
    print("perturbed golden", head_mode, errs)
    for k, v in errs.items():
        assert v < TOL, (k, errs)


@pytest.mark.gpu
def test_perturbed_full_view_indices_bit_exact(hip_lib, cuda):
    """512x512 perturbed view with parity weights: every ray's searchsorted
    indices and resampled bins of both proposal stages identical to the
    oracle's sample_pdf fed the kernels' weights and the same perturbed u;
    a seeded sample of rays end to end against the oracle."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, perturbed_positions
    H = W = 512
    N = H * W
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_params(spec, seed=34, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(W, H, rot=synth.random_rotation(3))
    ro, rd = ops.get_rays(pose, intr, H, W, device=cuda)
    torch.manual_seed(5)
    draws = perturbed_positions(N, list(spec.num_steps), cuda)
    out = FusedRenderer(net).render(ro, rd, taps=True, perturb=draws)
    torch.cuda.synchronize()
    o = {k: v.cpu().contiguous() for k, v in out.items()}
    d = [t.cpu() for t in draws]
    # stage 0 resamples the perturbed bins0 with u1, stage 1 bins1 with u2
    for st, (bins, w, T, gb, gi, u) in enumerate(((d[0], o["w0"], 65, o["bins1"], o["inds1"], d[1]),
                                                   (o["bins1"], o["w1"], 33, o["bins2"], o["inds2"], d[2]))):
        ref_b, ref_i = orc.sample_pdf(bins, w, T, return_inds=True, u=u)
        mism = (gi.long() != ref_i).sum().item()
        print(f"perturbed stage {st}: {mism} of {ref_i.numel()} indices differ")
        assert mism == 0
        assert torch.equal(gb, ref_b)
    idx = torch.from_numpy(np.random.default_rng(1).choice(N, 256, replace=False))
    ref = oracle_for(spec, params).run(ro.cpu()[idx], rd.cpu()[idx], return_feats=1,
                                       perturbed=tuple(t[idx] for t in d))
    errs = {k: (o[k][idx] - ref[k]).abs().max().item() for k in ("image", "weights_sum", "samvit")}
    errs["depth_rel"] = ((o["depth"][idx] - ref["depth"]).abs() / ref["depth"].abs().clamp(min=1.0)).max().item()
    print("perturbed 512x512 sampled rays", errs)
    for k, v in errs.items():
        assert v < TOL, (k, errs)
    assert torch.isfinite(o["samvit"]).all()


@pytest.mark.gpu
def test_run_perturb_fused_equals_run_torch(hip_lib, cuda):
    """NeRFRenderer.run(perturb=True) takes the fused path and draws on the
    device generator what run_torch(perturb=True) draws from the same seed,
    staged (per-chunk draws) as well; both differ from the unperturbed view."""
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    params = synth.make_params(spec, seed=22, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    from samnerf_amd import ops
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(4))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    net.opt.max_ray_batch = 1024
    with torch.no_grad():
        for staged in (False, True):
            torch.manual_seed(3)
            fused = net.render(ro, rd, staged=staged, perturb=True, return_feats=1)
            torch.manual_seed(3)
            if staged:
                ref = {}
                for h in range(0, ro.shape[0], 1024):
                    part = net.run_torch(ro[h:h + 1024], rd[h:h + 1024], perturb=True, return_feats=1)
                    for k, v in part.items():
                        ref.setdefault(k, []).append(v)
                ref = {k: torch.cat(v) for k, v in ref.items()}
            else:
                ref = net.run_torch(ro, rd, perturb=True, return_feats=1)
            errs = {k: (fused[k].reshape(ref[k].shape) - ref[k]).abs().max().item()
                    for k in ("image", "weights_sum", "samvit")}
            print("staged" if staged else "whole", errs)
            for k, v in errs.items():
                assert v < TOL, (k, errs)
        plain = net.render(ro, rd, staged=False, return_feats=1)
    assert (plain["image"] - fused["image"]).abs().max().item() > 1e-4      # the draw did act


@pytest.mark.gpu
def test_training_mode_teacher_render_is_fused(hip_lib, cuda):
    """The distillation step's teacher render (utils.py:1078-1079: train mode,
    no_grad, staged, perturb=True) runs on the fused kernels; with grad on,
    training mode stays on run_torch."""
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    params = synth.make_params(spec, seed=23, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda).train()
    ro = torch.zeros(256, 3, device=cuda)
    ro[:, 2] = 1.5
    rd = torch.nn.functional.normalize(torch.randn(256, 3, device=cuda, generator=torch.Generator(cuda).manual_seed(0)) * 0.2
                                       + torch.tensor([0.0, 0.0, -1.0], device=cuda), dim=-1)
    with torch.no_grad():
        assert net._fused_ok(ro, True, 0, {})
        torch.manual_seed(4)
        a = net.render(ro, rd, staged=True, perturb=True, update_proposal=False, return_feats=0)
        torch.manual_seed(4)
        b = net.run_torch(ro, rd, perturb=True, update_proposal=False, return_feats=0)
    assert (a["image"] - b["image"]).abs().max().item() < TOL
    assert not net._fused_ok(ro, True, 0, {})                 # grad enabled, train mode
