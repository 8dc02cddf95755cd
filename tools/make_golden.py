#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE's own Python code.

Runs only in the build container, where /root/reference exists (it never
travels to the GPU box; the tests read the committed .npz files).

What is imported from the reference (read-only, no bytecode written):
  nerf/renderer.py, nerf/network.py, encoding.py, activation.py and
  nerf/utils.py (for get_rays)
Third-party modules the reference imports at module level but does not use on
this path (cv2, mcubes, trimesh, torch_efficient_distloss, lpips, wandb, ...)
are replaced by inert stubs.  The reference's CUDA encoders (gridencoder /
shencoder / freqencoder) are NEVER imported -- their JIT build would write
into /root/reference -- instead `gridencoder.GridEncoder` and
`shencoder.SHEncoder` are stand-ins computing on the C oracle
(oracle/encoders_oracle.c), so the goldens pin everything except the encoder
kernels, which tests/test_oracle.py pins separately with KATs.

Each fixture stores inputs, outputs and the synth seed/config; parameters are
re-synthesised deterministically by oracle/synth.py.

usage: PYTHONDONTWRITEBYTECODE=1 python tools/make_golden.py
"""
import argparse
import importlib.machinery
import os
import sys
import types

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from oracle import encoders as enc  # noqa: E402
from oracle import renderer as orc  # noqa: E402
from oracle import synth  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")


# ------------------------------------------------------------------ stubs --

class _Anything:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Anything()

    def __getattr__(self, name):
        return _Anything()


class _StubModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _Anything()


def _stub(name):
    parts = name.split(".")
    for i in range(1, len(parts) + 1):
        n = ".".join(parts[:i])
        if n not in sys.modules:
            m = _StubModule(n)
            m.__spec__ = importlib.machinery.ModuleSpec(n, None)
            m.__path__ = []
            sys.modules[n] = m


TABLE_LOG2 = {}   # (num_levels, level_dim, desired) -> log2 override


class StandInGridEncoder(nn.Module):
    """Interface of gridencoder/grid.py:102-168, computing on the C oracle."""

    def __init__(self, input_dim=3, num_levels=16, level_dim=2, per_level_scale=2,
                 base_resolution=16, log2_hashmap_size=19, desired_resolution=None,
                 gridtype="hash", align_corners=False, interpolation="linear"):
        super().__init__()
        log2 = TABLE_LOG2.get((num_levels, level_dim, int(desired_resolution)), log2_hashmap_size)
        self.spec = synth.GridSpec(num_levels, level_dim, log2, int(desired_resolution),
                                   base_resolution, input_dim)
        offs = self.spec.offsets()
        self.register_buffer("offsets", torch.from_numpy(offs))
        self.embeddings = nn.Parameter(torch.zeros(int(offs[-1]), level_dim))
        self.output_dim = num_levels * level_dim
        self.input_dim = input_dim

    def forward(self, inputs, bound=1, max_level=None):
        inputs = (inputs + bound) / (2 * bound)
        prefix = list(inputs.shape[:-1])
        inputs = inputs.view(-1, self.input_dim)
        g = orc.OracleGrid(self.spec, self.embeddings.detach().numpy(), self.offsets.numpy())
        return g.encode01(inputs).view(prefix + [self.output_dim])


class StandInSHEncoder(nn.Module):
    """Interface of shencoder/sphere_harmonics.py:61-89 on the C oracle."""

    def __init__(self, input_dim=3, degree=4):
        super().__init__()
        self.input_dim, self.degree, self.output_dim = input_dim, degree, degree ** 2

    def forward(self, inputs, size=1):
        return orc.sh_encode(inputs / size * 1.0, self.degree) if size != 1 else orc.sh_encode(inputs, self.degree)


def install_reference():
    for n in ["cv2", "mcubes", "trimesh", "torch_efficient_distloss", "imageio", "tensorboardX",
              "wandb", "matplotlib", "matplotlib.pyplot", "torchmetrics",
              "torchmetrics.functional", "torch_ema", "lpips", "torchvision", "PIL",
              "dearpygui", "dearpygui.dearpygui"]:
        _stub(n)
    g = types.ModuleType("gridencoder")
    g.GridEncoder = StandInGridEncoder
    s = types.ModuleType("shencoder")
    s.SHEncoder = StandInSHEncoder
    sys.modules["gridencoder"] = g
    sys.modules["shencoder"] = s
    # the product package's directory (put on sys.path by oracle/synth.py)
    # holds a regular `nerf` package, which would win over the reference's
    # namespace package wherever it sits on the path
    sys.path[:] = [p for p in sys.path if not p.rstrip("/").endswith("segment-anything-nerf_amd")]
    sys.path.insert(0, REF)
    import importlib
    network = importlib.import_module("nerf.network")
    renderer = importlib.import_module("nerf.renderer")
    utils = importlib.import_module("nerf.utils")
    for mod in (network, renderer, utils):
        assert os.path.realpath(mod.__file__).startswith(REF + "/"), mod.__file__
    return network, renderer, utils


def make_opt(spec: synth.ModelSpec):
    return types.SimpleNamespace(
        bound=spec.bound, contract=True, min_near=spec.min_near, density_thresh=10,
        with_sam=spec.with_sam, sum_after_mlp=spec.sum_after_mlp, sam_use_view_direction=True,
        with_mask=spec.with_mask, mask_mlp_type=spec.mask_type,
        adaptive_mlp_type=spec.adaptive_type, num_steps=list(spec.num_steps),
        background="last_sample", max_ray_batch=4096 * 4, lambda_proposal=1,
        lambda_distort=0.02, fp16=False, n_inst=spec.n_inst,
        redundant_instance=spec.redundant_instance)


# -------------------------------------------------------------- fixtures --

def render_fixture(network, name, spec, seed, emb_scale, H, W, rot_seed, ln_jitter=0.1):
    TABLE_LOG2.clear()
    TABLE_LOG2[(16, 2, int(2048 * spec.grid_bound))] = spec.grid_log2
    assert not (spec.with_sam and spec.with_mask and spec.s_grid_log2 != spec.m_grid_log2)
    TABLE_LOG2[(16, 8, 512)] = spec.m_grid_log2 if spec.with_mask else spec.s_grid_log2
    TABLE_LOG2[(5, 2, 128)] = spec.prop_log2
    TABLE_LOG2[(5, 2, 256)] = spec.prop_log2
    params = synth.make_params(spec, seed=seed, emb_scale=emb_scale, ln_jitter=ln_jitter)
    model = network.NeRFNetwork(make_opt(spec))
    sd = model.state_dict()
    missing = [k for k in sd if k not in params]
    assert not missing, missing
    model.load_state_dict({k: torch.from_numpy(np.asarray(params[k])) for k in sd}, strict=True)
    model.eval()

    rot = synth.random_rotation(rot_seed) if rot_seed is not None else None
    pose, intr = synth.gui_camera(W, H, rot=rot)
    rays_o, rays_d = orc.get_rays(pose, intr, H, W)
    rm = int(spec.with_mask)
    with torch.no_grad():
        ref = model.run(rays_o, rays_d, return_feats=1, return_mask=rm, H=H, W=W)
    mine = orc.OracleNeRF(spec, params).run(rays_o, rays_d, return_feats=1, return_mask=rm, H=H, W=W)
    for k, v in ref.items():
        d = (v - mine[k]).abs().max().item()
        print(f"  {name}: {k:12s} max|ref-oracle| = {d:.3e}")
        assert d == 0.0, f"oracle restatement diverges from reference on {k}"
    out = dict(
        spec=np.array([spec.with_sam, spec.grid_log2, spec.s_grid_log2, spec.prop_log2], np.int64),
        mask_spec=np.array([spec.with_mask, spec.n_inst, spec.redundant_instance, spec.m_grid_log2,
                            spec.sum_after_mlp], np.int64),
        mask_types=np.array([spec.mask_type, spec.adaptive_type]),
        seed=np.int64(seed), emb_scale=np.float64(emb_scale), ln_jitter=np.float64(ln_jitter),
        pose=pose, intrinsics=intr, H=np.int64(H), W=np.int64(W),
        rays_o=rays_o.numpy(), rays_d=rays_d.numpy(),
        image=ref["image"].numpy(), depth=ref["depth"].numpy(),
        weights_sum=ref["weights_sum"].numpy())
    if spec.with_sam:
        out["samvit"] = ref["samvit"].reshape(H * W, -1).numpy()
    if spec.with_mask:
        out["instance_mask_logits"] = ref["instance_mask_logits"].numpy()
    np.savez_compressed(os.path.join(GOLDEN, name + ".npz"), **out)


def mask_fixtures(network):
    """--with_mask heads (network.py:125-203, renderer.py:392-454) in the
    configurations the reference's scripts run (scripts/train_mask.sh:
    adaptive + density + sum_after_mlp; scripts/test_mask_gui.sh: default +
    sum_after_mlp), plus the two head types whose reference forward raises:
    their exception types and messages are stored so the tests can require
    the same behaviour."""
    small = dict(grid_log2=12, s_grid_log2=11, prop_log2=10, m_grid_log2=11, with_sam=False)
    render_fixture(network, "render_mask_default",
                   synth.ModelSpec(with_mask=True, mask_type="default", sum_after_mlp=True, **small),
                   seed=7, emb_scale=0.5, H=16, W=16, rot_seed=6)
    render_fixture(network, "render_mask_default_nosum",
                   synth.ModelSpec(with_mask=True, mask_type="default", n_inst=3, redundant_instance=1,
                                   **small), seed=8, emb_scale=0.5, H=12, W=12, rot_seed=7)
    for at in ("density", "rgb"):
        render_fixture(network, f"render_mask_adaptive_{at}",
                       synth.ModelSpec(with_mask=True, mask_type="adaptive", adaptive_type=at,
                                       sum_after_mlp=True, **small),
                       seed=9, emb_scale=0.5, H=12, W=12, rot_seed=8)
    errs = {}
    for mt, at in (("lightweight_mask", "density"), ("adaptive", "sam")):
        spec = synth.ModelSpec(with_mask=True, mask_type=mt, adaptive_type=at, **small)
        TABLE_LOG2.clear()
        TABLE_LOG2[(16, 2, int(2048 * spec.grid_bound))] = spec.grid_log2
        TABLE_LOG2[(5, 2, 128)] = spec.prop_log2
        TABLE_LOG2[(5, 2, 256)] = spec.prop_log2
        params = synth.make_params(spec, seed=3, emb_scale=0.5)
        model = network.NeRFNetwork(make_opt(spec))
        model.load_state_dict({k: torch.from_numpy(np.asarray(params[k])) for k in model.state_dict()},
                              strict=True)
        model.eval()
        rays_o, rays_d = orc.get_rays(*synth.gui_camera(4, 4), 4, 4)
        try:
            with torch.no_grad():
                model.run(rays_o, rays_d, return_mask=1)
            raise AssertionError(f"{mt}/{at}: the reference did not raise")
        except (RuntimeError, AttributeError, TypeError) as e:
            errs[f"{mt}_{at}"] = (type(e).__name__, str(e).splitlines()[0][:200])
            print(f"  {mt}/{at}: reference raises {type(e).__name__}: {errs[f'{mt}_{at}'][1]}")
    np.savez_compressed(os.path.join(GOLDEN, "mask_errors.npz"),
                        **{k + "_type": np.array(v[0]) for k, v in errs.items()},
                        **{k + "_msg": np.array(v[1]) for k, v in errs.items()})


def perturbed_draws(N, steps, seed):
    """The random positions of run(perturb=True) drawn in the reference's order
    from torch.manual_seed(seed): renderer.py:268-271 (stage-0 bins), then
    sample_pdf's u (renderer.py:97-103) for stages 1 and 2 -- nothing else
    draws in between."""
    torch.manual_seed(seed)
    T0 = steps[0]
    bins = torch.linspace(0, 1, T0 + 1).unsqueeze(0).expand(N, -1)
    bins = (bins + (torch.rand_like(bins) - 0.5) / T0).clamp(0, 1)
    out = [bins.contiguous()]
    for T in (steps[1] + 1, steps[2] + 1):
        u = torch.linspace(0.5 / T, 1 - 0.5 / T, steps=T).expand(N, T)
        out.append((u + (torch.rand_like(u) - 0.5) / T).contiguous())
    return out


def perturbed_fixture(network):
    """run(perturb=True) of the reference (renderer.py:221-390 with the random
    sample positions of :268-271 and :100-101) on a 16x16 SAM view, from
    torch.manual_seed(11).  Stores the positions the draw produced, so the
    GPU path can be fed the same ones (the device generator draws others)."""
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=11, prop_log2=10)
    TABLE_LOG2.clear()
    TABLE_LOG2[(16, 2, int(2048 * spec.grid_bound))] = spec.grid_log2
    TABLE_LOG2[(16, 8, 512)] = spec.s_grid_log2
    TABLE_LOG2[(5, 2, 128)] = spec.prop_log2
    TABLE_LOG2[(5, 2, 256)] = spec.prop_log2
    params = synth.make_params(spec, seed=12, emb_scale=0.5, ln_jitter=0.1)
    model = network.NeRFNetwork(make_opt(spec))
    model.load_state_dict({k: torch.from_numpy(np.asarray(params[k])) for k in model.state_dict()},
                          strict=True)
    model.eval()
    H = W = 16
    pose, intr = synth.gui_camera(W, H, rot=synth.random_rotation(9))
    rays_o, rays_d = orc.get_rays(pose, intr, H, W)
    torch.manual_seed(11)
    with torch.no_grad():
        ref = model.run(rays_o, rays_d, perturb=True, return_feats=1, H=H, W=W)
    draws = perturbed_draws(H * W, list(spec.num_steps), 11)
    oracle = orc.OracleNeRF(spec, params)
    torch.manual_seed(11)
    mine = oracle.run(rays_o, rays_d, return_feats=1, H=H, W=W, perturb=True)
    given = oracle.run(rays_o, rays_d, return_feats=1, H=H, W=W, perturbed=draws)
    for k, v in ref.items():
        for other, what in ((mine, "perturb=True"), (given, "perturbed draws")):
            d = (v - other[k]).abs().max().item()
            print(f"  render_perturbed_sam: {k:12s} max|ref-oracle({what})| = {d:.3e}")
            assert d == 0.0, f"oracle restatement diverges from reference on {k} ({what})"
    np.savez_compressed(
        os.path.join(GOLDEN, "render_perturbed_sam.npz"),
        spec=np.array([spec.with_sam, spec.grid_log2, spec.s_grid_log2, spec.prop_log2], np.int64),
        seed=np.int64(12), emb_scale=np.float64(0.5), ln_jitter=np.float64(0.1), torch_seed=np.int64(11),
        pose=pose, intrinsics=intr, H=np.int64(H), W=np.int64(W),
        rays_o=rays_o.numpy(), rays_d=rays_d.numpy(),
        bins0=draws[0].numpy(), u1=draws[1].numpy(), u2=draws[2].numpy(),
        image=ref["image"].numpy(), depth=ref["depth"].numpy(),
        weights_sum=ref["weights_sum"].numpy(), samvit=ref["samvit"].reshape(H * W, -1).numpy())


def units_fixture(renderer, utils):
    g = torch.Generator().manual_seed(1234)
    out = {}
    # a1 get_rays (utils.py:145-279) for a rotated GUI camera
    pose, intr = synth.gui_camera(24, 16, rot=synth.random_rotation(7), center=(0.1, -0.2, 0.05))
    r = utils.get_rays(torch.from_numpy(pose)[None], torch.from_numpy(intr)[None], 16, 24, -1)
    out.update(rays_pose=pose, rays_intr=intr, rays_o=r["rays_o"].numpy(), rays_d=r["rays_d"].numpy())
    # a2 near/far incl. rays that miss the box (origin outside, pointing away)
    o = (torch.rand(512, 3, generator=g) - 0.5) * 2.0
    d = torch.randn(512, 3, generator=g)
    o[:32] = torch.tensor([200.0, 200.0, 0.0])      # outside, slab intervals disjoint
    d[:32] = torch.tensor([1.0, -1.0, 0.1])
    d[32:40, 1:] = 0.0                       # axis-aligned (1e-15 guard path)
    aabb = torch.tensor([-128.0] * 3 + [128.0] * 3)
    n, f = renderer.near_far_from_aabb(o, d, aabb, 0.2)
    out.update(nf_o=o.numpy(), nf_d=d.numpy(), nf_near=n.numpy(), nf_far=f.numpy())
    # a4 contract incl. |x|<1, ties and large magnitudes
    x = torch.randn(2048, 3, generator=g) * torch.tensor([0.3, 2.0, 50.0]).repeat_interleave(683)[:2048, None]
    x[:8] = torch.tensor([[1.5, -1.5, 0.2], [2.0, 2.0, 2.0], [-3.0, 1.0, 3.0], [0.5, 0.5, 0.5],
                          [1.0, 0.0, 0.0], [0.0, -1.0, 1.0], [1e6, 1.0, -1.0], [0.0, 0.0, 0.0]])
    out.update(contract_x=x.numpy(), contract_z=renderer.contract(x).numpy())
    # a5 sample_pdf for both resampling shapes, with degenerate rows
    for T0, T in [(128, 65), (64, 33)]:
        bins = torch.sort(torch.rand(256, T0 + 1, generator=g), -1).values
        w = torch.rand(256, T0, generator=g) ** 4
        w[0] = 0.0                            # all-zero weights -> uniform pdf
        w[1, :T0 // 2] = 0.0
        w[2, 5] = 1e6                         # spike -> cdf plateau at 1
        w[3] = torch.where(torch.rand(T0, generator=g) < 0.9, 0.0, 1.0)
        bins[4] = 0.5                         # zero-width bins
        nb = renderer.sample_pdf(bins, w, T, False)
        cdf_u = orc.sample_pdf(bins, w, T, return_inds=True)
        out[f"pdf{T0}_bins"] = bins.numpy()
        out[f"pdf{T0}_w"] = w.numpy()
        out[f"pdf{T0}_out"] = nb.numpy()
        out[f"pdf{T0}_inds_oracle"] = cdf_u[1].numpy()
        assert torch.equal(cdf_u[0], nb), "oracle sample_pdf diverges from reference"
    np.savez_compressed(os.path.join(GOLDEN, "units.npz"), **out)
    print("  units: written")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true")
    ap.add_argument("--only", choices=["perturbed"], help="write just this fixture")
    args = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)
    enc.build()
    network, renderer, utils = install_reference()
    if args.only == "perturbed":
        perturbed_fixture(network)
        return
    units_fixture(renderer, utils)
    small = dict(grid_log2=12, s_grid_log2=11, prop_log2=10)
    render_fixture(network, "render_small_rgb", synth.ModelSpec(with_sam=False, **small),
                   seed=1, emb_scale=0.5, H=16, W=16, rot_seed=3)
    render_fixture(network, "render_small_sam", synth.ModelSpec(with_sam=True, **small),
                   seed=2, emb_scale=0.5, H=16, W=16, rot_seed=4)
    render_fixture(network, "render_small_sam_default_init",
                   synth.ModelSpec(with_sam=True, **small),
                   seed=5, emb_scale=1e-4, H=8, W=8, rot_seed=None, ln_jitter=0.0)
    mask_fixtures(network)
    perturbed_fixture(network)
    if not args.skip_full:
        render_fixture(network, "render_full_sam", synth.ModelSpec(with_sam=True),
                       seed=3, emb_scale=0.5, H=8, W=8, rot_seed=5)


if __name__ == "__main__":
    main()
