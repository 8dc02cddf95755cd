"""Shared helpers for the parity tests."""
import numpy as np
import torch

from oracle import renderer as orc
from oracle import synth


def spec_from_fixture(fx):
    with_sam, g, s, p = [int(v) for v in fx["spec"]]
    return synth.ModelSpec(with_sam=bool(with_sam), grid_log2=g, s_grid_log2=s, prop_log2=p)


def make_net(spec, params, device):
    """The product's NeRFNetwork mirror loaded with synthesised parameters."""
    from nerf.network import NeRFNetwork, default_opt
    opt = default_opt(with_sam=spec.with_sam, grid_log2=spec.grid_log2,
                      s_grid_log2=spec.s_grid_log2, prop_log2=spec.prop_log2)
    net = NeRFNetwork(opt)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()},
                        strict=True)
    return net.to(device).eval()


def oracle_for(spec, params):
    return orc.OracleNeRF(spec, params)


def max_abs(a, b):
    a = a.detach().float().cpu() if torch.is_tensor(a) else torch.as_tensor(a)
    b = b.detach().float().cpu() if torch.is_tensor(b) else torch.as_tensor(b)
    return (a - b).abs().max().item()
