"""torch-CPU restatement of the reference renderer / network -- TEST INFRA ONLY.

Op-for-op restatement of
  nerf/utils.py:145-279      get_rays (full-image branch, N = -1)
  nerf/renderer.py:60-69     contract
  nerf/renderer.py:84-119    sample_pdf
  nerf/renderer.py:122-139   near_far_from_aabb
  nerf/renderer.py:185-219   render (staged chunking)
  nerf/renderer.py:221-390   run (sampling, compositing, SAM head)
  nerf/network.py:9-75       MLP / SkipConnMLP
  nerf/network.py:221-259    common_forward / forward / density
  activation.py:5-18         trunc_exp
with the encoders served by the C oracle (oracle/encoders_oracle.c).  Same torch
ops, same shapes, same order as the reference, so on the same inputs it agrees
bit for bit with the reference's own Python (pinned by tests/test_oracle.py
against tests/golden/*.npz made from the reference itself).
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import encoders as enc
from .synth import ModelSpec


# ------------------------------------------------------------- rays (a1) --

def get_rays(pose, intrinsics, H, W):
    """nerf/utils.py:145-279 with N=-1: pixel centres, camera dirs
    ((i-cx)/fx, -(j-cy)/fy, -1) not normalised, rotated by pose[:3,:3]."""
    poses = torch.as_tensor(np.asarray(pose, np.float32)).view(1, 4, 4)
    intr = torch.as_tensor(np.asarray(intrinsics, np.float32)).view(1, 4)
    fx, fy, cx, cy = intr[:, 0], intr[:, 1], intr[:, 2], intr[:, 3]
    i, j = torch.meshgrid(torch.linspace(0, W - 1, W), torch.linspace(0, H - 1, H),
                          indexing="ij")
    i = i.t().contiguous().view(-1) + 0.5
    j = j.t().contiguous().view(-1) + 0.5
    zs = -torch.ones_like(i)
    xs = (i - cx) / fx
    ys = -(j - cy) / fy
    directions = torch.stack((xs, ys, zs), dim=-1)
    rays_d = (directions.unsqueeze(1) @ poses[:, :3, :3].transpose(-1, -2)).squeeze(1)
    rays_o = poses[:, :3, 3].expand_as(rays_d)
    return rays_o.contiguous(), rays_d.contiguous()


# ------------------------------------------------------ free functions --

def near_far_from_aabb(rays_o, rays_d, aabb, min_near=0.05):
    """nerf/renderer.py:122-139 (no-hit sentinel 1e9, near >= min_near)."""
    tmin = (aabb[:3] - rays_o) / (rays_d + 1e-15)
    tmax = (aabb[3:] - rays_o) / (rays_d + 1e-15)
    near = torch.where(tmin < tmax, tmin, tmax).amax(dim=-1, keepdim=True)
    far = torch.where(tmin > tmax, tmin, tmax).amin(dim=-1, keepdim=True)
    mask = far < near
    near[mask] = 1e9
    far[mask] = 1e9
    near = torch.clamp(near, min=min_near)
    return near, far


def contract(x):
    """nerf/renderer.py:60-69: L-inf contraction to [-2, 2]."""
    shape, C = x.shape[:-1], x.shape[-1]
    x = x.view(-1, C)
    mag, idx = x.abs().max(1, keepdim=True)
    scale = 1 / mag.repeat(1, C)
    scale.scatter_(1, idx, (2 - 1 / mag) / mag)
    z = torch.where(mag < 1, x, x * scale)
    return z.view(*shape, C)


def sample_pdf(bins, weights, T, perturb=False, return_inds=False, u=None):
    """nerf/renderer.py:84-119 (inverse-CDF resampling).  `u` [N, T]: given
    sample positions (a perturbed draw made beforehand) instead of lines
    97-103's."""
    N, T0 = weights.shape
    weights = weights + 0.01
    weights_sum = torch.sum(weights, -1, keepdim=True)
    pdf = weights / weights_sum
    cdf = torch.cumsum(pdf, -1).clamp(max=1)
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    if u is None:
        u = torch.linspace(0.5 / T, 1 - 0.5 / T, steps=T).to(weights.device)
        u = u.expand(N, T)
        if perturb:
            u = u + (torch.rand_like(u) - 0.5) / T
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = torch.clamp(inds - 1, 0, T0)
    above = torch.clamp(inds, 0, T0)
    cdf_g0 = torch.gather(cdf, -1, below)
    cdf_g1 = torch.gather(cdf, -1, above)
    bins_g0 = torch.gather(bins, -1, below)
    bins_g1 = torch.gather(bins, -1, above)
    bins_t = torch.clamp(torch.nan_to_num((u - cdf_g0) / (cdf_g1 - cdf_g0)), 0, 1)
    out = bins_g0 + bins_t * (bins_g1 - bins_g0)
    return (out, inds) if return_inds else out


def spacing_fn(x):
    return torch.where(x < 1, x / 2, 1 - 1 / (2 * x))


def spacing_fn_inv(x):
    return torch.where(x < 0.5, 2 * x, 1 / (2 - 2 * x))


def composite_weights(real_bins, sigmas, last_sample=True):
    """nerf/renderer.py:310-326: sigmas -> weights."""
    deltas = (real_bins[..., 1:] - real_bins[..., :-1])
    deltas_sigmas = deltas * sigmas
    return composite_from_ds(deltas_sigmas, last_sample)


def composite_from_ds(deltas_sigmas, last_sample=True):
    """nerf/renderer.py:312-326, from the optical depths deltas * sigmas on
    (the parity taps of the fused path hand these over, samnerf_set_taps)."""
    if last_sample:
        deltas_sigmas = torch.cat(
            [deltas_sigmas[..., :-1], torch.full_like(deltas_sigmas[..., -1:], torch.inf)], dim=-1)
    alphas = 1 - torch.exp(-deltas_sigmas)
    transmittance = torch.cumsum(deltas_sigmas[..., :-1], dim=-1)
    transmittance = torch.cat([torch.zeros_like(transmittance[..., :1]), transmittance], dim=-1)
    transmittance = torch.exp(-transmittance)
    weights = alphas * transmittance
    weights.nan_to_num_(0)
    return weights


# ------------------------------------------------------------ encoders --

class OracleGrid:
    """GridEncoder(...).forward (gridencoder/grid.py:151-168) on the C oracle."""

    def __init__(self, spec, embeddings, offsets):
        self.spec = spec
        self.embeddings = np.ascontiguousarray(embeddings, np.float32)
        self.offsets = np.ascontiguousarray(offsets, np.int32)
        self.L = spec.num_levels
        self.C = spec.level_dim
        self.S = np.log2(spec.per_level_scale)
        self.H = spec.base_resolution

    def encode01(self, x01):
        """[B,3] in [0,1] -> [B, L*C] (grid.py:60-63 incl. the permute)."""
        out = enc.grid_encode_forward(x01.detach().cpu().numpy(), self.embeddings,
                                      self.offsets, self.L, self.S, self.H)
        t = torch.from_numpy(out)
        return t.permute(1, 0, 2).reshape(x01.shape[0], self.L * self.C)

    def __call__(self, inputs, bound=1):
        inputs = (inputs + bound) / (2 * bound)
        prefix = list(inputs.shape[:-1])
        inputs = inputs.reshape(-1, 3)
        return self.encode01(inputs).view(prefix + [self.L * self.C])


def sh_encode(d, degree=4):
    """SHEncoder.forward (shencoder/sphere_harmonics.py:75-89)."""
    d = d / 1
    d = d / torch.norm(d, dim=-1, keepdim=True)
    prefix = list(d.shape[:-1])
    out = enc.sh_encode_forward(d.reshape(-1, 3).numpy(), degree)
    return torch.from_numpy(out).reshape(prefix + [degree * degree])


# ---------------------------------------------------------------- model --

def mlp(x, weights, ir=None):
    """MLP.forward (nerf/network.py:23-34), bias-free, ReLU between layers;
    `ir` (a list) receives each layer's output after its activation, as
    save_intermedian_results stores them (network.py:32-33)."""
    for l, W in enumerate(weights):
        x = F.linear(x, W)
        if l != len(weights) - 1:
            x = F.relu(x, inplace=True)
        if ir is not None:
            ir.append(x.detach())
    return x


def skip_mlp(x, layers, skip_layers=(2,)):
    """SkipConnMLP.forward (nerf/network.py:63-75): leaky_relu(0.01)."""
    x_in = x
    for l, (W, b) in enumerate(layers):
        if l in skip_layers:
            x = torch.cat([x, x_in], dim=-1)
        x = F.linear(x, W, b)
        if l != len(layers) - 1:
            x = F.leaky_relu(x, inplace=True)
    return x


class OracleNeRF:
    """NeRFNetwork(opt) (nerf/network.py:94-259) + NeRFRenderer.run/render."""

    def __init__(self, spec: ModelSpec, params):
        self.spec = spec
        t = lambda k: torch.from_numpy(np.ascontiguousarray(params[k]))
        self.grid = OracleGrid(spec.grid, params["grid.embeddings"], params["grid.offsets"])
        self.grid_mlp = [t(f"grid_mlp.net.{i}.weight") for i in range(3)]
        self.view_mlp = [t(f"view_mlp.net.{i}.weight") for i in range(3)]
        self.prop_grids = [OracleGrid(g, params[f"prop_encoders.{i}.embeddings"],
                                      params[f"prop_encoders.{i}.offsets"])
                           for i, g in enumerate(spec.prop)]
        self.prop_mlp = [[t(f"prop_mlp.{i}.net.0.weight"), t(f"prop_mlp.{i}.net.1.weight")]
                         for i in range(len(spec.prop))]
        if spec.with_sam:
            self.s_grid = OracleGrid(spec.s_grid, params["s_grid.embeddings"],
                                     params["s_grid.offsets"])
            self.sam_layers = [(t(f"samvit_mlp.0.net.{i}.weight"), t(f"samvit_mlp.0.net.{i}.bias"))
                               for i in range(5)]
            self.ln_w = t("samvit_mlp.1.weight")
            self.ln_b = t("samvit_mlp.1.bias")
        if spec.with_mask:
            if spec.m_grid is not None:
                self.m_grid = OracleGrid(spec.m_grid, params["m_grid.embeddings"],
                                         params["m_grid.offsets"])
            self.mask_w = [t(name + ".weight") for name, _, _, _ in spec.mask_shapes()]
        self.aabb = t("aabb_infer")
        self.bound = spec.grid_bound

    # network.py:221-229
    def common_forward(self, x, ir=None):
        grid_output = self.grid(x, bound=self.bound)
        f = mlp(grid_output, self.grid_mlp, ir)
        sigma = torch.exp(f[..., 0])              # trunc_exp forward, activation.py:15-18
        feat = f[..., 1:]
        return sigma, feat, grid_output

    # network.py:231-246
    def forward(self, x, d, ir=None):
        sigma, feat, grid_output = self.common_forward(x, ir)
        d = sh_encode(d, self.spec.sh_degree)
        f_color = torch.cat([feat, d], dim=-1)
        return {"sigma": sigma, "geo_feat": feat, "color": f_color, "grid_output": grid_output}

    # network.py:248-259
    def density(self, x, proposal=-1):
        if 0 <= proposal < len(self.prop_grids):
            sigma = torch.exp(mlp(self.prop_grids[proposal](x, bound=self.bound),
                                  self.prop_mlp[proposal]).squeeze(-1))
        else:
            sigma, _, _ = self.common_forward(x)
        return {"sigma": sigma}

    @torch.no_grad()
    def stage_sigmas(self, rays_o, rays_d, bins, stage):
        """One stage of renderer.py:250-300 at GIVEN bins [N, T+1] (the fused
        path's own, read through its parity taps): real bins (:250-265),
        sample positions (:276-281), contract, then network.density with
        proposal=stage (network.py:248-259) for stages 0-1 or common_forward's
        sigma (network.py:221-229) for the final stage.  Returns sigmas
        [N, T], deltas * sigmas [N, T] (renderer.py:310-311, the last sample's
        as computed, before :313-315 replaces it by inf), real_bins
        [N, T+1] and the grid-space positions (x + bound) / (2 bound)
        [N, T, 3] (grid.py:156)."""
        rays_o = rays_o.contiguous()
        rays_d = rays_d.contiguous()
        nears, fars = near_far_from_aabb(rays_o, rays_d, self.aabb, self.spec.min_near)
        s_nears = spacing_fn(nears)
        s_fars = spacing_fn(fars)
        real_bins = spacing_fn_inv(s_nears * (1 - bins) + s_fars * bins)
        rays_t = (real_bins[..., 1:] + real_bins[..., :-1]) / 2
        xyzs = rays_o.unsqueeze(1) + rays_d.unsqueeze(1) * rays_t.unsqueeze(2)
        xyzs = contract(xyzs)
        if stage < len(self.prop_grids):
            sigmas = self.density(xyzs, proposal=stage)["sigma"]
        else:
            sigmas, _, _ = self.common_forward(xyzs)
        deltas = real_bins[..., 1:] - real_bins[..., :-1]
        return sigmas, deltas * sigmas, real_bins, (xyzs + self.bound) / (2 * self.bound)

    def sam_head(self, f):
        """samvit_mlp = Sequential(SkipConnMLP(163,256,256,5,skip=[2]), LayerNorm(256))."""
        x = skip_mlp(f, self.sam_layers)
        return F.layer_norm(x, (256,), self.ln_w, self.ln_b, 1e-5)

    def mask_head(self, masks, outputs, colors, grid_ir, view_ir):
        """Per-sample instance logits, renderer.py:392-452."""
        spec, M = self.spec, self.mask_w
        if spec.mask_type == "default":
            return skip_mlp(torch.cat([masks, outputs["geo_feat"].detach()], dim=-1),
                            [(W, None) for W in M], skip_layers=())
        if spec.mask_type == "lightweight_mask":       # 63 inputs into a 35-input MLP: raises, as the reference
            return mlp(torch.cat([masks, colors.detach()], dim=-1), M)
        g = grid_ir
        if spec.adaptive_type == "rgb":
            v = view_ir
            m = F.linear(outputs["grid_output"].detach(), M[0])
            m = F.linear(torch.cat([g[0], m], dim=-1), M[1])
            m = F.linear(torch.cat([g[1], m], dim=-1), M[2])
            m = F.linear(torch.cat([g[2], m], dim=-1), M[3])
            m = F.linear(torch.cat([v[0], m], dim=-1), M[4])
            m = F.linear(torch.cat([v[1], m], dim=-1), M[5])
            m = F.linear(m, M[6])
            return F.linear(m, M[7])
        if spec.adaptive_type == "density":
            m = F.linear(outputs["grid_output"].detach(), M[0])
            m = F.linear(torch.cat([g[0], m], dim=-1), M[1])
            m = F.linear(torch.cat([g[1], m], dim=-1), M[2])
            m = F.linear(torch.cat([g[2], m], dim=-1), M[3])
            m = F.linear(m, M[4])
            return F.linear(m, M[5])
        raise AttributeError("'Sequential' object has no attribute 'intermedian_reuslts' "
                             "(renderer.py:448: the reference's adaptive 'sam' head reads "
                             "intermediates its samvit_mlp never stores)")

    @torch.no_grad()
    def run(self, rays_o, rays_d, bg_color=None, return_feats=0, return_mask=0, H=None, W=None,
            keep=None, perturb=False, perturbed=None):
        """nerf/renderer.py:221-464 in eval mode (contract=True,
        background='last_sample', sam_use_view_direction; sum_after_mlp for
        the RGB + mask configurations).  `keep` (a dict) receives per-stage
        intermediates for finer checks.  perturb=True draws torch.rand_like
        where the reference does (renderer.py:268-271, :100-101); `perturbed`
        = (bins0 [N, T0+1], u1 [N, T1+1], u2 [N, T2+1]) supplies those
        positions instead (the same draw made beforehand)."""
        rays_o = rays_o.contiguous()
        rays_d = rays_d.contiguous()
        N = rays_o.shape[0]
        nears, fars = near_far_from_aabb(rays_o, rays_d, self.aabb, self.spec.min_near)
        if bg_color is None:
            bg_color = 1
        results = {}
        s_nears = spacing_fn(nears)
        s_fars = spacing_fn(fars)
        bins = weights = None
        steps = self.spec.num_steps
        for prop_iter in range(len(steps)):
            if prop_iter == 0:
                bins = torch.linspace(0, 1, steps[prop_iter] + 1).unsqueeze(0)
                bins = bins.expand(N, -1)
                if perturbed is not None:
                    bins = perturbed[0]
                elif perturb:
                    bins = bins + (torch.rand_like(bins) - 0.5) / (steps[prop_iter])
                    bins = bins.clamp(0, 1)
            else:
                u = perturbed[prop_iter] if perturbed is not None else None
                bins = sample_pdf(bins, weights, steps[prop_iter] + 1, perturb, u=u).detach()
            real_bins = spacing_fn_inv(s_nears * (1 - bins) + s_fars * bins)
            rays_t = (real_bins[..., 1:] + real_bins[..., :-1]) / 2
            xyzs = rays_o.unsqueeze(1) + rays_d.unsqueeze(1) * rays_t.unsqueeze(2)
            xyzs = contract(xyzs)
            if prop_iter != len(steps) - 1:
                sigmas = self.density(xyzs, proposal=prop_iter)["sigma"]
            else:
                dirs = rays_d.view(-1, 1, 3).expand_as(xyzs)
                dirs = dirs / torch.norm(dirs, dim=-1, keepdim=True)
                grid_ir = []
                outputs = self.forward(xyzs, dirs, grid_ir)
                sigmas = outputs["sigma"]
                colors = outputs["color"]
                if self.spec.with_sam:
                    features = self.s_grid(xyzs, bound=self.bound)
                if return_mask > 0 and self.spec.mask_type in ("default", "lightweight_mask"):
                    masks = self.m_grid(xyzs, bound=self.bound)
            weights = composite_weights(real_bins, sigmas)
            if keep is not None:
                if prop_iter < len(steps) - 1 and perturbed is not None:
                    keep[f"u{prop_iter}"] = perturbed[prop_iter + 1]
                keep[f"bins{prop_iter}"] = bins.clone()
                keep[f"weights{prop_iter}"] = weights.clone()
                keep[f"sigmas{prop_iter}"] = sigmas.clone()
        weights_sum = torch.sum(weights, dim=-1)
        depth = torch.sum(weights * rays_t, dim=-1)
        f_image = torch.sum(weights.unsqueeze(-1) * colors, dim=-2)
        view_ir = []
        if self.spec.sum_after_mlp:                      # renderer.py:339-342
            f_colors = mlp(colors, self.view_mlp, view_ir)
            image = torch.sigmoid(torch.sum(weights.unsqueeze(-1) * f_colors, dim=-2))
        else:
            image = torch.sigmoid(mlp(f_image, self.view_mlp, view_ir))
        image = image + (1 - weights_sum).unsqueeze(-1) * bg_color
        results["weights_sum"] = weights_sum
        results["depth"] = depth
        results["image"] = image
        if self.spec.with_sam:
            if self.spec.sum_after_mlp:
                raise NotImplementedError("with_sam + sum_after_mlp: the reference's branch "
                                          "crashes (renderer.py:371-372, SURVEY.md 0.2)")
            f_sam = torch.sum(weights.unsqueeze(-1) * features, dim=-2)
            f = torch.cat([f_sam, f_image, image, depth.unsqueeze(-1)], dim=-1)
            samvit = self.sam_head(f)
            if keep is not None:
                keep["f_sam"] = f_sam
                keep["f_image"] = f_image
            if return_feats > 0:
                results["samvit"] = samvit.view(H, W, -1) if H is not None else samvit
        if return_mask > 0:                              # renderer.py:392-454
            point_masks = self.mask_head(masks if self.spec.mask_type in ("default", "lightweight_mask")
                                         else None, outputs, colors, grid_ir, view_ir)
            results["instance_mask_logits"] = torch.sum(weights.detach().unsqueeze(-1) * point_masks,
                                                        dim=-2)
        return results

    def render(self, rays_o, rays_d, max_ray_batch=4096 * 4, **kw):
        """nerf/renderer.py:185-219 (staged); samvit rows stay flat [N,256]."""
        N = rays_o.shape[0]
        out = {}
        for head in range(0, N, max_ray_batch):
            r = self.run(rays_o[head:head + max_ray_batch], rays_d[head:head + max_ray_batch], **kw)
            for k, v in r.items():
                out.setdefault(k, []).append(v.reshape(v.shape[0], -1) if k == "samvit" else v)
        return {k: torch.cat(v, 0) for k, v in out.items()}
