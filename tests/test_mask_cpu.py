"""--with_mask instance heads (nerf/network.py:125-203,
nerf/renderer.py:392-454) on the CPU: the product's NeRFNetwork mirror runs its
unfused path (run_torch) with the C oracle's encoders swapped in
(tests/oracle_backend.py), so everything but the encoder kernels is the
product's own code; it must reproduce the goldens made by the reference's
Python bit for bit, and raise where the reference raises."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from helpers import fixture_params, make_net, spec_from_fixture
from oracle import renderer as orc
from oracle import synth
from oracle_backend import oracle_encoders

MASK_FIXTURES = ["render_mask_default", "render_mask_default_nosum", "render_mask_adaptive_density",
                 "render_mask_adaptive_rgb"]


@pytest.mark.parametrize("name", MASK_FIXTURES)
def test_mirror_mask_heads_match_reference_golden(oracle_lib, name):
    fx = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec = spec_from_fixture(fx)
    net = make_net(spec, fixture_params(fx, spec), "cpu")
    ro, rd = torch.from_numpy(fx["rays_o"]), torch.from_numpy(fx["rays_d"])
    with oracle_encoders(), torch.no_grad():
        out = net.render(ro, rd, staged=True, return_mask=1)        # run_torch (no fused path on CPU)
    for k in ("image", "depth", "weights_sum", "instance_mask_logits"):
        assert np.array_equal(out[k].numpy(), fx[k]), (k, float((out[k] - torch.from_numpy(fx[k])).abs().max()))


@pytest.mark.parametrize("mt,at", [("lightweight_mask", "density"), ("adaptive", "sam")])
def test_broken_reference_heads_raise_like_the_reference(oracle_lib, mt, at):
    errs = np.load(os.path.join(GOLDEN, "mask_errors.npz"))
    etype = str(errs[f"{mt}_{at}_type"])
    spec = synth.ModelSpec(with_sam=False, with_mask=True, mask_type=mt, adaptive_type=at,
                           grid_log2=12, prop_log2=10, m_grid_log2=11)
    net = make_net(spec, synth.make_params(spec, seed=3, emb_scale=0.5), "cpu")
    ro, rd = orc.get_rays(*synth.gui_camera(4, 4), 4, 4)
    exc = {"RuntimeError": RuntimeError, "AttributeError": AttributeError}[etype]
    with oracle_encoders(), torch.no_grad(), pytest.raises(exc):
        net.run_torch(ro, rd, return_mask=1)


def test_mask_state_dict_keys_are_the_references():
    """Checkpoint compatibility: the mirror's mask-head parameters carry the
    reference's state_dict names and shapes (strict load of the synthesised
    reference-shaped dicts)."""
    for mt, at in [("default", "density"), ("lightweight_mask", "density"), ("adaptive", "rgb"),
                   ("adaptive", "density"), ("adaptive", "sam")]:
        spec = synth.ModelSpec(with_sam=at == "sam", with_mask=True, mask_type=mt, adaptive_type=at,
                               grid_log2=10, s_grid_log2=10, prop_log2=9, m_grid_log2=10)
        net = make_net(spec, synth.make_params(spec, seed=1), "cpu")       # load_state_dict(strict=True)
        groups = net.get_params(1e-2)
        n = sum(p.numel() for g in groups for p in g["params"])
        assert n == sum(p.numel() for p in net.parameters()), (mt, at)
