"""Deterministic synthesis of model parameters, camera poses and rays.

Shared by the golden generator (tools/make_golden.py), the tests and bench.py
so that fixtures only need to store a seed + config, never 200 MB of tables.

Architecture and defaults follow the reference:
  * hash grids:    nerf/network.py:102 (grid), :111 (s_grid), :211/:216 (proposals)
  * table layout:  gridencoder/grid.py:106-135 (offsets from double-precision
                   ceil(base * scale**l), rounded up to a multiple of 8)
  * MLPs:          nerf/network.py:103, :107, :120-123, :212/:217
  * camera:        nerf/gui.py:10-45 (OrbitCamera pose / intrinsics), main.py:203-208
Initialisation mirrors torch's defaults in distribution (nn.Linear
U(+-1/sqrt(fan_in)); embeddings U(+-1e-4), grid.py:144-146) but draws from a
numpy PCG64 stream per named tensor so every process gets identical bits.
"""
import math
import zlib
from dataclasses import dataclass, field

import numpy as np


@dataclass
class GridSpec:
    """One GridEncoder(input_dim=3, ...) as nerf/network.py instantiates it."""
    num_levels: int
    level_dim: int
    log2_hashmap_size: int
    desired_resolution: int
    base_resolution: int = 16
    input_dim: int = 3

    @property
    def per_level_scale(self):
        # grid.py:107-108
        return float(np.exp2(np.log2(self.desired_resolution / self.base_resolution)
                             / (self.num_levels - 1)))

    @property
    def S(self):
        # grid.py:38: S = np.log2(per_level_scale), handed to the kernel as float
        return float(np.log2(self.per_level_scale))

    def offsets(self):
        # grid.py:124-135
        offs, o = [], 0
        max_params = 2 ** self.log2_hashmap_size
        for i in range(self.num_levels):
            res = int(np.ceil(self.base_resolution * self.per_level_scale ** i))
            n = min(max_params, res ** self.input_dim)
            n = int(np.ceil(n / 8) * 8)
            offs.append(o)
            o += n
        offs.append(o)
        return np.array(offs, dtype=np.int32)

    @property
    def output_dim(self):
        return self.num_levels * self.level_dim


@dataclass
class ModelSpec:
    """NeRFNetwork(opt) with main.py's forced settings (main.py:222-226):
    contract=True -> grid bound 2, bound=128 -> aabb +-128."""
    with_sam: bool = True
    bound: float = 128.0
    grid_bound: float = 2.0
    min_near: float = 0.2
    num_steps: tuple = (128, 64, 32)
    # log2 table sizes; the reference hard-codes 19 / 19 / 17 / 17
    grid_log2: int = 19
    s_grid_log2: int = 19
    prop_log2: int = 17
    geo_feat_dim: int = 15
    sh_degree: int = 4
    # --with_mask heads (nerf/network.py:125-203; main.py:112-148 defaults)
    with_mask: bool = False
    mask_type: str = "default"          # default | lightweight_mask | adaptive
    adaptive_type: str = "density"      # rgb | density | sam (adaptive only)
    n_inst: int = 2
    redundant_instance: int = 0
    m_grid_log2: int = 19
    sum_after_mlp: bool = False
    extras: dict = field(default_factory=dict)

    @property
    def grid(self):
        return GridSpec(16, 2, self.grid_log2, int(2048 * self.grid_bound))

    @property
    def s_grid(self):
        return GridSpec(16, 8, self.s_grid_log2, 512)

    @property
    def prop(self):
        return [GridSpec(5, 2, self.prop_log2, 128), GridSpec(5, 2, self.prop_log2, 256)]

    @property
    def m_grid(self):
        """network.py:127-128 (default) / :138-139 (lightweight_mask); the
        lightweight table size is hard-coded to 2^10 in the reference."""
        if not self.with_mask or self.mask_type == "adaptive":
            return None
        if self.mask_type == "default":
            return GridSpec(16, 8, self.m_grid_log2, 512)
        return GridSpec(16, 2, 10, 256)

    def mask_shapes(self):
        """(name, out, in, bias) of the mask head's Linears (network.py:125-203)."""
        if not self.with_mask:
            return []
        g, sh = self.geo_feat_dim, self.sh_degree ** 2
        n_out = self.n_inst + self.redundant_instance
        if self.mask_type == "default":                  # SkipConnMLP(143, n_out, 256, 3), bias off
            m = self.m_grid.output_dim + g
            return [("mask_mlp.0.net.0", 256, m, False), ("mask_mlp.0.net.1", 256, 256, False),
                    ("mask_mlp.0.net.2", n_out, 256, False)]
        if self.mask_type == "lightweight_mask":         # MLP(15 + 16 + 4, n_out, 64, 3)
            return [("mask_mlp.net.0", 64, g + sh + 4, False), ("mask_mlp.net.1", 64, 64, False),
                    ("mask_mlp.net.2", n_out, 64, False)]
        d = 96                                           # adaptive: bias-free Linears
        ins = {"rgb": [(d, 32), (d, 64 + d), (d, 64 + d), (d, 16 + d), (d, 32 + d), (d, 32 + d),
                       (d, d), (self.n_inst, d)],
               "density": [(d, 32), (d, 64 + d), (d, 64 + d), (d, 16 + d), (d, d), (self.n_inst, d)],
               "sam": [(32, 64), (32, 64 + 32), (64, 16 + 32), (256, 256 + 64), (256, 512),
                       (256, 512), (self.n_inst, 512)]}[self.adaptive_type]
        return [(f"mask_mlp.{i}", o, i_, False) for i, (o, i_) in enumerate(ins)]

    def linear_shapes(self):
        """(name, out, in, bias) in state_dict order of the reference modules."""
        g = self.geo_feat_dim
        sh = self.sh_degree ** 2
        shapes = [
            ("grid_mlp.net.0", 64, self.grid.output_dim, False),
            ("grid_mlp.net.1", 64, 64, False),
            ("grid_mlp.net.2", 1 + g, 64, False),
            ("view_mlp.net.0", 32, g + sh, False),
            ("view_mlp.net.1", 32, 32, False),
            ("view_mlp.net.2", 3, 32, False),
        ]
        if self.with_sam:
            din = self.s_grid.output_dim + g + sh + 4          # 163, network.py:121
            shapes += [
                ("samvit_mlp.0.net.0", 256, din, True),
                ("samvit_mlp.0.net.1", 256, 256, True),
                ("samvit_mlp.0.net.2", 256, 256 + din, True),  # skip layer 2
                ("samvit_mlp.0.net.3", 256, 256, True),
                ("samvit_mlp.0.net.4", 256, 256, True),
            ]
        shapes += self.mask_shapes()
        for i, p in enumerate(self.prop):
            shapes += [(f"prop_mlp.{i}.net.0", 16, p.output_dim, False),
                       (f"prop_mlp.{i}.net.1", 1, 16, False)]
        return shapes


def _rng(seed, name):
    return np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(name.encode())]))


def uniform(seed, name, shape, lo, hi):
    r = _rng(seed, name).random(int(np.prod(shape)), dtype=np.float64)
    return (lo + (hi - lo) * r).astype(np.float32).reshape(shape)


def make_params(spec: ModelSpec, seed=0, emb_scale=1e-4, ln_jitter=0.0):
    """State-dict-shaped numpy parameters (keys as in the reference)."""
    P = {}
    grids = [("grid", spec.grid)]
    if spec.with_sam:
        grids.append(("s_grid", spec.s_grid))
    if spec.m_grid is not None:
        grids.append(("m_grid", spec.m_grid))
    grids += [(f"prop_encoders.{i}", g) for i, g in enumerate(spec.prop)]
    for name, g in grids:
        offs = g.offsets()
        P[f"{name}.offsets"] = offs
        P[f"{name}.embeddings"] = uniform(seed, name, (int(offs[-1]), g.level_dim),
                                          -emb_scale, emb_scale)
    for name, o, i, has_bias in spec.linear_shapes():
        k = 1.0 / math.sqrt(i)
        P[f"{name}.weight"] = uniform(seed, name + ".weight", (o, i), -k, k)
        if has_bias:
            P[f"{name}.bias"] = uniform(seed, name + ".bias", (o,), -k, k)
    if spec.with_sam:
        P["samvit_mlp.1.weight"] = (1.0 + uniform(seed, "ln.w", (256,), -ln_jitter, ln_jitter)
                                    ).astype(np.float32)
        P["samvit_mlp.1.bias"] = uniform(seed, "ln.b", (256,), -ln_jitter, ln_jitter)
    aabb = np.array([-spec.bound] * 3 + [spec.bound] * 3, np.float32)
    P["aabb_train"] = aabb
    P["aabb_infer"] = aabb.copy()
    return P


def gui_camera(W=512, H=512, radius=0.5, fovy=60.0, rot=None, center=(0.0, 0.0, 0.0)):
    """Pose [4,4] and intrinsics (fx, fy, cx, cy) exactly as OrbitCamera builds
    them (nerf/gui.py:24-45).  `rot` is an optional 3x3 rotation."""
    res = np.eye(4, dtype=np.float32)
    res[2, 3] = radius
    r4 = np.eye(4, dtype=np.float32)
    if rot is not None:
        r4[:3, :3] = np.asarray(rot, np.float32)
    pose = r4 @ res
    pose[:3, 3] -= np.asarray(center, np.float32)
    focal = H / (2 * np.tan(np.radians(fovy) / 2))
    intr = np.array([focal, focal, W // 2, H // 2], dtype=np.float32)
    return pose.astype(np.float32), intr


def random_rotation(seed):
    """Seeded uniform rotation (QR of a Gaussian matrix, sign-fixed)."""
    g = _rng(seed, "rotation").standard_normal((3, 3))
    q, r = np.linalg.qr(g)
    q = q * np.sign(np.diag(r))
    if np.linalg.det(q) < 0:
        q[:, 0] = -q[:, 0]
    return q.astype(np.float32)


def _level_resolutions(g: GridSpec):
    """Indexing resolution per level (float32 formula of gridencoder.cu:133)."""
    S32 = np.float32(g.S)
    return [int(np.ceil(np.float32(np.exp2(np.float32(l) * S32)) * np.float32(g.base_resolution)))
            for l in range(g.num_levels)]


def _sphere_channel(g: GridSpec, table, bound, radius, amp):
    """Channel 0 of the dense levels of `table` = +amp at the vertices inside a
    sphere of `radius` (contracted units, at the origin), -amp outside; hashed
    levels' channel 0 = 0.  Returns the dense level indices."""
    offs = g.offsets()
    dense = []
    for l, res in enumerate(_level_resolutions(g)):
        n = int(offs[l + 1] - offs[l])
        if res ** 3 > n:                                  # hashed level (gridencoder.cu:61-79)
            table[offs[l]:offs[l + 1], 0] = 0.0
            continue
        dense.append(l)
        i = np.arange(res, dtype=np.float64)
        x = ((i + 0.5) / res) * 2 * bound - bound          # vertex i sits at u = (i + 0.5) / res
        X, Y, Z = np.meshgrid(x, x, x, indexing="ij")      # row = ix + iy res + iz res^2
        inside = (X * X + Y * Y + Z * Z) < radius * radius
        ch = np.where(inside, amp, -amp).astype(np.float32).transpose(2, 1, 0).reshape(-1)
        table[offs[l]:offs[l] + res ** 3, 0] = ch
    return dense


def make_surface_params(spec: ModelSpec, seed=0, radius=0.3, amp=1.5, emb_scale=0.5, ln_jitter=0.1):
    """make_params plus an opaque sphere: a scene whose rays saturate (the
    trained-scene regime random weights never reach: there the transmittance
    stays above 1e-2 until the last sample).  The density grid's and the
    proposal grids' dense levels carry +-amp in channel 0 (inside / outside
    the sphere), and the first rows of grid_mlp / prop_mlp route that channel
    to the density output (two ReLU units for the positive and negative parts,
    so the raw density is +amp * levels inside and -amp * levels outside).
    Used by the flagged early-exit mode's tests and bench line (N1)."""
    P = make_params(spec, seed=seed, emb_scale=emb_scale, ln_jitter=ln_jitter)
    b = spec.grid_bound

    def route(w0, w1, w2, dense, C):
        cols = [l * C for l in dense]
        w0[0, :] = 0.0
        w0[1, :] = 0.0
        w0[0, cols] = 1.0
        w0[1, cols] = -1.0
        if w2 is None:                                     # prop_mlp: 2 layers, 1 output
            w1[0, :] = 0.0
            w1[0, 0], w1[0, 1] = 1.0, -1.0
            return
        w1[0:2, :] = 0.0
        w1[0, 0] = 1.0
        w1[1, 1] = 1.0
        w2[0, :] = 0.0
        w2[0, 0], w2[0, 1] = 1.0, -1.0

    d = _sphere_channel(spec.grid, P["grid.embeddings"], b, radius, amp)
    route(P["grid_mlp.net.0.weight"], P["grid_mlp.net.1.weight"], P["grid_mlp.net.2.weight"], d,
          spec.grid.level_dim)
    for i, g in enumerate(spec.prop):
        d = _sphere_channel(g, P[f"prop_encoders.{i}.embeddings"], b, radius, amp)
        route(P[f"prop_mlp.{i}.net.0.weight"], P[f"prop_mlp.{i}.net.1.weight"], None, d, g.level_dim)
    return P
