"""Shared helpers for the parity tests."""
import numpy as np
import torch

from oracle import renderer as orc
from oracle import synth


def spec_from_fixture(fx):
    with_sam, g, s, p = [int(v) for v in fx["spec"]]
    kw = {}
    if "mask_spec" in fx:
        with_mask, n_inst, red, m_log2, sum_after = [int(v) for v in fx["mask_spec"]]
        mt, at = [str(v) for v in fx["mask_types"]]
        kw = dict(with_mask=bool(with_mask), n_inst=n_inst, redundant_instance=red,
                  m_grid_log2=m_log2, sum_after_mlp=bool(sum_after), mask_type=mt, adaptive_type=at)
    return synth.ModelSpec(with_sam=bool(with_sam), grid_log2=g, s_grid_log2=s, prop_log2=p, **kw)


def fixture_params(fx, spec):
    return synth.make_params(spec, seed=int(fx["seed"]), emb_scale=float(fx["emb_scale"]),
                             ln_jitter=float(fx["ln_jitter"]))


def make_opt(spec):
    from nerf.network import default_opt
    return default_opt(with_sam=spec.with_sam, grid_log2=spec.grid_log2,
                       s_grid_log2=spec.s_grid_log2, prop_log2=spec.prop_log2,
                       with_mask=spec.with_mask, mask_mlp_type=spec.mask_type,
                       adaptive_mlp_type=spec.adaptive_type, n_inst=spec.n_inst,
                       redundant_instance=spec.redundant_instance, m_grid_log2=spec.m_grid_log2,
                       sum_after_mlp=spec.sum_after_mlp)


def make_net(spec, params, device):
    """The product's NeRFNetwork mirror loaded with synthesised parameters."""
    from nerf.network import NeRFNetwork
    opt = make_opt(spec)
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
