"""NeRFNetwork on gfx950 -- interface of nerf/network.py:9-308.

Same submodules, parameter names and shapes as the reference (checkpoint
state_dicts load with strict=True), including the --with_mask instance heads
(network.py:125-203: 'default', 'lightweight_mask', 'adaptive' with
'rgb' / 'density' / 'sam').
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from activation import trunc_exp
from encoding import get_encoder

from .renderer import NeRFRenderer


class MLP(nn.Module):
    """network.py:9-34: Linear (+ReLU between layers)."""

    def __init__(self, dim_in, dim_out, dim_hidden, num_layers, bias=True):
        super().__init__()
        self.dim_in, self.dim_out, self.dim_hidden, self.num_layers = dim_in, dim_out, dim_hidden, num_layers
        self.net = nn.ModuleList([
            nn.Linear(dim_in if l == 0 else dim_hidden,
                      dim_out if l == num_layers - 1 else dim_hidden, bias=bias)
            for l in range(num_layers)])

    def forward(self, x, save_intermedian_results=True):
        """network.py:23-34: `intermedian_reuslts` (the reference's attribute
        name) keeps each layer's detached output after its activation; the
        adaptive mask heads read them (renderer.py:403-451)."""
        if save_intermedian_results:
            self.intermedian_reuslts = []
        for l, layer in enumerate(self.net):
            x = layer(x)
            if l != self.num_layers - 1:
                x = F.relu(x, inplace=True)
            if save_intermedian_results:
                self.intermedian_reuslts.append(x.detach())
        return x


class SkipConnMLP(nn.Module):
    """network.py:36-75: Linear + leaky_relu(0.01), input re-concatenated at
    the skip layers."""

    def __init__(self, dim_in, dim_out, dim_hidden, num_layers, skip_layers=(), bias=True):
        super().__init__()
        self.dim_in, self.dim_out, self.dim_hidden, self.num_layers = dim_in, dim_out, dim_hidden, num_layers
        self.skip_layers = list(skip_layers)
        layers = []
        for l in range(num_layers):
            fin = dim_in if l == 0 else (dim_hidden + dim_in if l in self.skip_layers else dim_hidden)
            fout = dim_out if l == num_layers - 1 else dim_hidden
            layers.append(nn.Linear(fin, fout, bias=bias))
        self.net = nn.ModuleList(layers)

    def forward(self, x, save_intermedian_results=False):
        x_in = x
        if save_intermedian_results:
            self.intermedian_reuslts = []
        for l, layer in enumerate(self.net):
            if l in self.skip_layers:
                x = torch.cat([x, x_in], dim=-1)
            x = layer(x)
            if l != self.num_layers - 1:
                x = F.leaky_relu(x, inplace=True)
            if save_intermedian_results:
                self.intermedian_reuslts.append(x.detach())
        return x


class NeRFNetwork(NeRFRenderer):
    def __init__(self, opt):
        super().__init__(opt)
        self.geom_feat_dim = 15
        # table sizes are hard-coded in the reference (19 / 19 / 17); the
        # optional opt.*_log2 overrides exist for small-table test fixtures
        g_log2 = getattr(opt, "grid_log2", 19)
        s_log2 = getattr(opt, "s_grid_log2", 19)
        p_log2 = getattr(opt, "prop_log2", 17)
        self.grid, self.grid_in_dim = get_encoder("hashgrid", input_dim=3, level_dim=2,
                                                  num_levels=16, log2_hashmap_size=g_log2,
                                                  desired_resolution=2048 * self.bound)
        self.grid_mlp = MLP(self.grid_in_dim, 1 + self.geom_feat_dim, 64, 3, bias=False)
        self.view_encoder, self.view_in_dim = get_encoder("sh", input_dim=3, degree=4)
        self.view_mlp = MLP(self.geom_feat_dim + self.view_in_dim, 3, 32, 3, bias=False)
        if opt.with_sam:
            self.s_grid, self.s_dim = get_encoder("hashgrid", input_dim=3, num_levels=16,
                                                  level_dim=8, base_resolution=16,
                                                  log2_hashmap_size=s_log2, desired_resolution=512)
            self.samvit_mlp = nn.Sequential(
                SkipConnMLP(self.s_dim + self.geom_feat_dim + self.view_in_dim + 4, 256, 256, 5,
                            skip_layers=[2], bias=True),
                nn.LayerNorm(256))
        if getattr(opt, "with_mask", False):
            self._build_mask_head(opt)
        self.prop_encoders = nn.ModuleList()
        self.prop_mlp = nn.ModuleList()
        for desired in (128, 256):
            enc, dim = get_encoder("hashgrid", input_dim=3, level_dim=2, num_levels=5,
                                   log2_hashmap_size=p_log2, desired_resolution=desired)
            self.prop_encoders.append(enc)
            self.prop_mlp.append(MLP(dim, 1, 16, 2, bias=False))

    def _build_mask_head(self, opt):
        """network.py:125-203."""
        n_out = opt.n_inst + getattr(opt, "redundant_instance", 0)
        mtype = opt.mask_mlp_type
        if mtype == "default":
            self.m_grid, self.m_dim = get_encoder(
                "hashgrid", input_dim=3, num_levels=16, level_dim=8, base_resolution=16,
                log2_hashmap_size=getattr(opt, "m_grid_log2", 19), desired_resolution=512)
            self.mask_mlp = nn.Sequential(SkipConnMLP(self.m_dim + self.geom_feat_dim, n_out, 256, 3,
                                                      skip_layers=[], bias=False))
        elif mtype == "lightweight_mask":
            self.m_grid, self.m_dim = get_encoder(
                "hashgrid", input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                log2_hashmap_size=10, desired_resolution=256)
            self.mask_mlp = MLP(self.geom_feat_dim + self.view_in_dim + 4, n_out, 64, 3, bias=False)
        elif mtype == "adaptive":
            d = self.mask_mlp_dim = 96
            at = opt.adaptive_mlp_type
            shapes = {"rgb": [(self.grid_in_dim, d), (64 + d, d), (64 + d, d), (16 + d, d),
                              (32 + d, d), (32 + d, d), (d, d), (d, opt.n_inst)],
                      "density": [(self.grid_in_dim, d), (64 + d, d), (64 + d, d), (16 + d, d),
                                  (d, d), (d, opt.n_inst)],
                      "sam": [(64, 32), (64 + 32, 32), (16 + 32, 64), (256 + 64, 256), (256 + 256, 256),
                              (256 + 256, 256), (256 + 256, opt.n_inst)]}[at]
            self.mask_mlp = nn.ModuleList([nn.Linear(i, o, bias=False) for i, o in shapes])
        else:
            raise ValueError(f"unknown mask_mlp_type {mtype!r}")

    def mask_logits(self, masks, outputs, colors):
        """Per-sample instance logits (renderer.py:392-452)."""
        mtype = self.opt.mask_mlp_type
        if mtype == "default":
            return self.mask_mlp(torch.cat([masks, outputs["geo_feat"].detach()], dim=-1))
        if mtype == "lightweight_mask":     # 63 inputs into a 35-input MLP: raises, like the reference
            return self.mask_mlp(torch.cat([masks, colors.detach()], dim=-1))
        M, g = self.mask_mlp, self.grid_mlp.intermedian_reuslts
        at = self.opt.adaptive_mlp_type
        if at == "rgb":
            v = self.view_mlp.intermedian_reuslts
            m = M[0](outputs["grid_output"].detach())
            m = M[1](torch.cat([g[0], m], dim=-1))
            m = M[2](torch.cat([g[1], m], dim=-1))
            m = M[3](torch.cat([g[2], m], dim=-1))
            m = M[4](torch.cat([v[0], m], dim=-1))
            m = M[5](torch.cat([v[1], m], dim=-1))
            return M[7](M[6](m))
        if at == "density":
            m = M[0](outputs["grid_output"].detach())
            m = M[1](torch.cat([g[0], m], dim=-1))
            m = M[2](torch.cat([g[1], m], dim=-1))
            m = M[3](torch.cat([g[2], m], dim=-1))
            return M[5](M[4](m))
        s = self.samvit_mlp.intermedian_reuslts      # AttributeError, as in the reference
        m = M[0](g[0])
        m = M[1](torch.cat([g[1], m], dim=-1))
        m = M[2](torch.cat([g[2], m], dim=-1))
        m = M[3](torch.cat([s[0], m], dim=-1))
        m = M[4](torch.cat([s[1], m], dim=-1))
        m = M[5](torch.cat([s[2], m], dim=-1))
        return M[6](torch.cat([s[3], m], dim=-1))

    def common_forward(self, x, save_intermedian_results=False):
        grid_output = self.grid(x, bound=self.bound)
        f = self.grid_mlp(grid_output, save_intermedian_results)
        return trunc_exp(f[..., 0]), f[..., 1:], grid_output

    def forward(self, x, d, save_intermedian_results=False, **kwargs):
        sigma, feat, grid_output = self.common_forward(x, save_intermedian_results)
        d = self.view_encoder(d)
        return {"sigma": sigma, "geo_feat": feat, "color": torch.cat([feat, d], dim=-1),
                "grid_output": grid_output}

    def density(self, x, proposal=-1):
        if 0 <= proposal < len(self.prop_encoders):
            h = self.prop_encoders[proposal](x, bound=self.bound)
            sigma = trunc_exp(self.prop_mlp[proposal](h).squeeze(-1))
        else:
            sigma, _, _ = self.common_forward(x)
        return {"sigma": sigma}

    def _reg_grid(self):
        """network.py:261-275: the grid the TV / weight-decay regularisers act on."""
        if self.opt.with_sam:
            return self.s_grid
        if getattr(self.opt, "with_mask", False):
            return self.m_grid
        return self.grid

    def apply_total_variation(self, w):
        self._reg_grid().grad_total_variation(w)

    def apply_weight_decay(self, w):
        self._reg_grid().grad_weight_decay(w)

    def get_params(self, lr):
        params = [{"params": self.grid.parameters(), "lr": lr},
                  {"params": self.grid_mlp.parameters(), "lr": lr},
                  {"params": self.view_mlp.parameters(), "lr": lr},
                  {"params": self.prop_encoders.parameters(), "lr": lr},
                  {"params": self.prop_mlp.parameters(), "lr": lr}]
        if self.opt.with_sam:
            params += [{"params": self.s_grid.parameters(), "lr": lr},
                       {"params": self.samvit_mlp.parameters(), "lr": lr}]
        if getattr(self.opt, "with_mask", False):
            if self.opt.mask_mlp_type in ("default", "lightweight_mask"):
                params.append({"params": self.m_grid.parameters(), "lr": lr})
            params.append({"params": self.mask_mlp.parameters(), "lr": lr})
        return params


def default_opt(with_sam=True, **kw):
    """The option namespace NeRFNetwork reads, with main.py's defaults and its
    forced overrides (main.py:222-226: fp16 off, bound 128, contract on)."""
    import types
    o = dict(bound=128.0, contract=True, min_near=0.2, density_thresh=10, with_sam=with_sam,
             sum_after_mlp=False, sam_use_view_direction=True, with_mask=False,
             mask_mlp_type="default", adaptive_mlp_type="density", n_inst=2, redundant_instance=0,
             epsilon=1e-6,
             num_steps=[128, 64, 32], background="last_sample", max_ray_batch=4096 * 4, fp16=False,
             # training (main.py:75-110, 226)
             lr=1e-2, num_rays=4096, adaptive_num_rays=True, num_points=2 ** 18,
             lambda_entropy=0.0, lambda_tv=0.0, lambda_wd=0.0, lambda_proposal=1.0,
             lambda_distort=0.02)
    o.update(kw)
    return types.SimpleNamespace(**o)
