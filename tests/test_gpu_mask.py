"""--with_mask instance heads on the MI355X: the mirror's
unfused path with the HIP drop-in encoders against the reference goldens
(1e-3), and the mask training step (nerf/utils.py:941-977) reducing its loss."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from helpers import fixture_params, make_net, spec_from_fixture
from oracle import synth

pytestmark = pytest.mark.gpu

MASK_FIXTURES = ["render_mask_default", "render_mask_default_nosum", "render_mask_adaptive_density",
                 "render_mask_adaptive_rgb"]


@pytest.mark.parametrize("name", MASK_FIXTURES)
def test_mask_heads_match_reference_golden(hip_lib, cuda, name):
    fx = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec = spec_from_fixture(fx)
    net = make_net(spec, fixture_params(fx, spec), cuda)
    ro = torch.from_numpy(fx["rays_o"]).to(cuda)
    rd = torch.from_numpy(fx["rays_d"]).to(cuda)
    with torch.no_grad():
        out = net.render(ro, rd, staged=True, return_mask=1)
    for k in ("image", "weights_sum", "instance_mask_logits"):
        err = (out[k].cpu() - torch.from_numpy(fx[k])).abs().max().item()
        assert err < 1e-3, (k, err)
    d_ref = torch.from_numpy(fx["depth"])
    assert ((out["depth"].cpu() - d_ref).abs() / d_ref.abs().clamp(min=1.0)).max() < 1e-3


def test_mask_training_reduces_loss(hip_lib, cuda):
    from samnerf_amd.train import mask_train_step
    spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="default", sum_after_mlp=True,
                           grid_log2=12, prop_log2=10, m_grid_log2=12)
    net = make_net(spec, synth.make_params(spec, seed=5, emb_scale=0.5), cuda).train()
    for k, p in net.named_parameters():              # main.py:255-262: only the mask head trains
        p.requires_grad = k.startswith("m_grid") or k.startswith("mask_mlp")
    opt = torch.optim.Adam([p for p in net.parameters() if p.requires_grad], lr=1e-2, eps=1e-15)
    pose, intr = synth.gui_camera(32, 32, rot=synth.random_rotation(3))
    from samnerf_amd import ops
    ro, rd = ops.get_rays(pose, intr, 32, 32, device=cuda)
    gt = (torch.arange(32 * 32, device=cuda) % 32 >= 16).long()     # right half = instance 1
    losses = []
    for _ in range(12):
        _, loss = mask_train_step(net, ro, rd, gt)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert losses[-1] < 0.5 * losses[0], losses


@pytest.mark.parametrize("head_mode", [0, 1])
@pytest.mark.parametrize("name", ["render_mask_default_nosum", "render_mask_default"])
def test_fused_mask_head_matches_reference_golden(hip_lib, cuda, monkeypatch, name, head_mode):
    """The 'default' mask head (m_grid L16C8 + SkipConnMLP 143->256->256->K) on
    the fused kernels: render(..., return_mask=1) takes k_final<GEO> (+ SA for
    the sum_after_mlp fixture: the view MLP per sample) + k_mask_head
    (mask_head.hip) and matches the reference's own golden within 1e-3, in
    both precision modes."""
    fx = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec = spec_from_fixture(fx)
    net = make_net(spec, fixture_params(fx, spec), cuda)
    net.head_mode = head_mode                        # the fused path's GEMM precision
    ro = torch.from_numpy(fx["rays_o"]).to(cuda)
    rd = torch.from_numpy(fx["rays_d"]).to(cuda)
    with torch.no_grad():
        out = net.render(ro, rd, staged=False, return_mask=1)
    assert net._fused is not None and net._fused.fused_mask_ok()          # the fused path ran
    for k in ("image", "weights_sum", "instance_mask_logits"):
        err = (out[k].cpu() - torch.from_numpy(fx[k])).abs().max().item()
        print(head_mode, k, err)
        assert err < 1e-3, (k, err)


@pytest.mark.parametrize("head_mode", [0, 1])
def test_fused_mask_head_matches_unfused_path(hip_lib, cuda, head_mode):
    """Full-size m_grid (2^19 rows), 5 instances: the fused mask logits against
    the unfused op sequence (torch GEMMs + HIP encoders) on a 64 x 64 view; the
    tiled render (view_width) gives the same bits as row-major waves."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="default", n_inst=3,
                           redundant_instance=2, sum_after_mlp=False)
    net = make_net(spec, synth.make_params(spec, seed=12, emb_scale=0.5), cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(8))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    fr = FusedRenderer(net, head_mode=head_mode)
    with torch.no_grad():
        ref = net.run_torch(ro, rd, return_mask=1)["instance_mask_logits"]
        got = fr.render(ro, rd, mask=True)["instance_mask_logits"]
        tiled = fr.render(ro, rd, mask=True, view_width=64)["instance_mask_logits"]
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    print("fused mask vs unfused", head_mode, err, scale)
    assert got.shape == (64 * 64, 5)
    assert err < 1e-3 * max(1.0, scale), (err, scale)
    assert torch.equal(got, tiled)
    # ragged launches: a partial last workgroup (4019 = 31 x 128 + 51 rays) and a
    # single part-filled one (5 rays) give each ray the bits of the full launch
    # (a ray's logits depend on that ray only; the weight ring runs regardless)
    with torch.no_grad():
        for n in (4019, 5):
            sub = fr.render(ro[:n], rd[:n], mask=True)["instance_mask_logits"]
            assert torch.equal(sub, got[:n]), n


def test_fused_sum_after_mlp_rgb_matches_unfused(hip_lib, cuda, monkeypatch, diag):
    """--sum_after_mlp on an RGB model (image = sigmoid(sum_k w_k
    view_mlp(colour_k)), renderer.py:339-342) on the fused k_final<SA> against
    the unfused op sequence, all segment forms (S = 1 / 2 / 4 by ray count)."""
    from samnerf_amd import ops
    spec = synth.ModelSpec(with_sam=False, sum_after_mlp=True)
    net = make_net(spec, synth.make_params(spec, seed=14, emb_scale=0.5), cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(5))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    with torch.no_grad():
        ref = net.run_torch(ro, rd)
        for seg, n in ((1, 4096), (2, 4096), (4, 1000)):
            monkeypatch.setenv("SAMNERF_FINAL_S", str(seg))
            out = net.run(ro[:n], rd[:n])
            assert net._fused is not None
            for k in ("image", "weights_sum"):
                err = (out[k] - ref[k][:n]).abs().max().item()
                assert err < 1e-3, (seg, n, k, err)


@pytest.mark.parametrize("name", ["render_mask_adaptive_density", "render_mask_adaptive_rgb"])
def test_fused_adaptive_mask_heads_match_reference_golden(hip_lib, cuda, name):
    """The 'adaptive' heads (bias-free Linear chains on the grid_mlp / view_mlp
    intermediates) on the fused path: k_final<..., AD> accumulates the
    weighted per-sample inputs, k_mask_eff multiplies the chain out; the
    reference's goldens within 1e-3 (both fixtures use sum_after_mlp)."""
    fx = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec = spec_from_fixture(fx)
    net = make_net(spec, fixture_params(fx, spec), cuda)
    ro = torch.from_numpy(fx["rays_o"]).to(cuda)
    rd = torch.from_numpy(fx["rays_d"]).to(cuda)
    with torch.no_grad():
        out = net.render(ro, rd, staged=False, return_mask=1)
    assert net._fused is not None and net._fused.fused_mask_ok()
    for k in ("image", "weights_sum", "instance_mask_logits"):
        err = (out[k].cpu() - torch.from_numpy(fx[k])).abs().max().item()
        print(name, k, err)
        assert err < 1e-3, (k, err)


@pytest.mark.parametrize("sum_after", [False, True])
def test_fused_adaptive_density_matches_unfused_path(hip_lib, cuda, sum_after):
    """Adaptive 'density' head at full table size, with and without
    sum_after_mlp, against the unfused op sequence on a 64 x 64 view."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="adaptive", adaptive_type="density",
                           n_inst=4, sum_after_mlp=sum_after)
    net = make_net(spec, synth.make_params(spec, seed=13, emb_scale=0.5), cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(9))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    with torch.no_grad():
        ref = net.run_torch(ro, rd, return_mask=1)
        got = FusedRenderer(net).render(ro, rd, mask=True, view_width=64)
    for k in ("image", "instance_mask_logits"):
        err = (got[k] - ref[k]).abs().max().item()
        scale = ref[k].abs().max().item()
        print("adaptive density", sum_after, k, err, scale)
        assert err < 1e-3 * max(1.0, scale), (k, err, scale)


@pytest.mark.parametrize("kind", ["default", "adaptive_density", "adaptive_rgb_sum"])
def test_mask_models_final_layout_bit_identical(hip_lib, cuda, monkeypatch, diag, kind):
    """Mask models on k_final's compile-time layout of the reference grid (LAY 1:
    the 'default' head's geo_feat form at S = 1, the adaptive heads' weighted-sum
    forms) against the run-time layout (SAMNERF_FINAL_LAY=0): image, depth,
    weights_sum and the instance logits bit for bit, on 70,000 rays of a
    512-wide view (S = 1), the form under test asserted by samnerf_last_forms."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, last_forms
    if kind == "default":
        spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="default", n_inst=2,
                               sum_after_mlp=False)
    elif kind == "adaptive_density":
        spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="adaptive",
                               adaptive_type="density", n_inst=4, sum_after_mlp=False)
    else:
        spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type="adaptive",
                               adaptive_type="rgb", n_inst=4, sum_after_mlp=True)
    net = make_net(spec, synth.make_params(spec, seed=17, emb_scale=0.5), cuda)
    pose, intr = synth.gui_camera(512, 160, rot=synth.random_rotation(21))
    ro, rd = ops.get_rays(pose, intr, 160, 512, device=cuda)
    n = 70000
    fr = FusedRenderer(net)
    outs = []
    for lay in ("0", "1"):
        monkeypatch.setenv("SAMNERF_FINAL_LAY", lay)
        with torch.no_grad():
            o = fr.render(ro[:n], rd[:n], mask=True)
        assert last_forms()[2] == int(lay)
        outs.append({k: v.cpu() for k, v in o.items() if torch.is_tensor(v)})
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
