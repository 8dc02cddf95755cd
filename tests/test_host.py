"""Host-side logic of the product package (CPU only): module interfaces,
state_dict compatibility with the reference layout, table geometry."""
import numpy as np
import pytest
import torch

from oracle import synth


def test_network_state_dict_matches_reference_layout():
    from nerf.network import NeRFNetwork, default_opt
    net = NeRFNetwork(default_opt(with_sam=True))
    sd = net.state_dict()
    params = synth.make_params(synth.ModelSpec(with_sam=True), emb_scale=1e-4)
    assert set(sd) == set(params)
    for k, v in params.items():
        assert tuple(sd[k].shape) == tuple(np.asarray(v).shape), k
    for g in ("grid", "s_grid", "prop_encoders.0", "prop_encoders.1"):
        assert np.array_equal(sd[f"{g}.offsets"].numpy(), params[f"{g}.offsets"])
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()}, strict=True)
    assert sum(p.numel() for p in net.parameters()) == 56_651_728


def test_rgb_only_network():
    from nerf.network import NeRFNetwork, default_opt
    net = NeRFNetwork(default_opt(with_sam=False))
    assert not hasattr(net, "s_grid")
    assert sum(p.numel() for p in net.parameters()) == 14_236_240


def test_grid_encoder_interface():
    from gridencoder import GridEncoder
    g = GridEncoder(input_dim=3, num_levels=16, level_dim=8, base_resolution=16,
                    log2_hashmap_size=19, desired_resolution=512)
    assert g.output_dim == 128 and g.embeddings.shape == (5258512, 8)
    assert "GridEncoder:" in repr(g)
    assert abs(g.embeddings.detach()).max() <= 1e-4
    with pytest.raises(ValueError, match="grad is None"):
        g.grad_weight_decay(0.1)


def test_encoder_factory():
    from encoding import get_encoder
    e, d = get_encoder("sh", degree=4)
    assert d == 16
    e, d = get_encoder("frequency", multires=6)
    assert d == 3 + 3 * 2 * 6
    e, d = get_encoder("frequency_torch", multires=4)
    x = torch.rand(5, 3)
    assert e(x).shape == (5, d)
    e, d = get_encoder("tiledgrid", num_levels=4, level_dim=2, desired_resolution=64)
    assert e.gridtype_id == 1 and d == 8
    with pytest.raises(NotImplementedError):
        get_encoder("nope")


def test_trunc_exp_forward_backward():
    from activation import trunc_exp
    x = torch.tensor([-20.0, 0.0, 3.0, 20.0], requires_grad=True)
    y = trunc_exp(x)
    y.sum().backward()
    assert torch.allclose(y, torch.exp(x))
    assert torch.allclose(x.grad, torch.exp(x.detach().clamp(-15, 15)))


def test_shard_range_partitions_exactly():
    from samnerf_amd.dist import shard_range
    for n in (0, 1, 7, 262144, 262147):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_surface_scene_is_an_opaque_sphere():
    """synth.make_surface_params (the N1 scene): the density of the main
    network and of both proposal networks is large inside the sphere and
    small outside (oracle evaluation, CPU)."""
    import torch
    from oracle import renderer as orc
    from samnerf_amd import synth
    spec = synth.ModelSpec(with_sam=False, grid_log2=16, prop_log2=15)
    net = orc.OracleNeRF(spec, synth.make_surface_params(spec, seed=1, radius=0.3, amp=1.5))
    inside = torch.tensor([[0.0, 0.0, 0.0], [0.1, -0.1, 0.05]])
    outside = torch.tensor([[0.8, 0.0, 0.0], [0.0, -0.9, 0.3]])
    for p in (-1, 0, 1):
        s_in = net.density(inside, proposal=p)["sigma"]
        s_out = net.density(outside, proposal=p)["sigma"]
        assert bool((s_in > 20).all()) and bool((s_out < 0.05).all()), (p, s_in, s_out)


def test_ray_of_slots_matches_ray_tiles():
    """fused.ray_of_slots restates RayTiles (samnerf_common.h): a permutation
    of the view's pixels, 8 x 4 tiles in row-major tile order; the identity
    where the tiling does not apply."""
    import torch
    from samnerf_amd.fused import ray_of_slots
    W, H = 64, 16
    m = ray_of_slots(W * H, W)
    assert torch.equal(torch.sort(m).values, torch.arange(W * H))
    for s in (0, 1, 7, 8, 31, 32, 33, 255, 256, W * H - 1):
        tile, inn = s // 32, s % 32
        trow, tcol = tile // (W // 8), tile % (W // 8)
        assert int(m[s]) == (trow * 4 + inn // 8) * W + tcol * 8 + inn % 8
    assert torch.equal(ray_of_slots(W * H - W, W), torch.arange(W * H - W))   # not 4 whole rows
    assert torch.equal(ray_of_slots(100, 0), torch.arange(100))
