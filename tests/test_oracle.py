"""Pin the CPU oracle (CPU-only; no GPU).

* against golden vectors produced by the reference's own Python
  (tools/make_golden.py imports nerf/renderer.py + nerf/network.py);
* against reference-independent known answers for the encoder kernels the
  goldens cannot cover (the reference's .cu cannot run here): SciPy real
  spherical harmonics, F.grid_sample trilinear on dense levels, literal
  hash vectors, adjointness of the grid backward, closed forms for WD / freq.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN
from oracle import encoders as enc
from oracle import renderer as orc
from oracle import synth


from helpers import spec_from_fixture as _spec_from  # noqa: E402

RENDER_FIXTURES = ["render_small_rgb", "render_small_sam", "render_small_sam_default_init",
                   "render_full_sam", "render_mask_default", "render_mask_default_nosum",
                   "render_mask_adaptive_density", "render_mask_adaptive_rgb"]


@pytest.mark.parametrize("name", RENDER_FIXTURES)
def test_oracle_render_matches_reference_golden(oracle_lib, name):
    fx = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec = _spec_from(fx)
    params = synth.make_params(spec, seed=int(fx["seed"]), emb_scale=float(fx["emb_scale"]),
                               ln_jitter=float(fx["ln_jitter"]))
    H, W = int(fx["H"]), int(fx["W"])
    ro, rd = orc.get_rays(fx["pose"], fx["intrinsics"], H, W)
    assert np.array_equal(ro.numpy(), fx["rays_o"]) and np.array_equal(rd.numpy(), fx["rays_d"])
    out = orc.OracleNeRF(spec, params).run(ro, rd, return_feats=1, return_mask=int(spec.with_mask),
                                           H=H, W=W)
    for k in ("image", "depth", "weights_sum"):
        assert np.array_equal(out[k].numpy(), fx[k]), k
    if spec.with_sam:
        assert np.array_equal(out["samvit"].reshape(H * W, -1).numpy(), fx["samvit"])
    if spec.with_mask:
        assert np.array_equal(out["instance_mask_logits"].numpy(), fx["instance_mask_logits"])


@pytest.mark.parametrize("name", ["render_small_sam", "render_small_rgb"])
def test_stage_sigmas_restates_run(oracle_lib, name):
    """OracleNeRF.stage_sigmas (the per-sample sigma checker of the GPU
    parity tests) at run()'s own bins gives run()'s sigmas and weights bit for
    bit, so it carries run()'s pin to the reference goldens (above)."""
    fx = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec = _spec_from(fx)
    params = synth.make_params(spec, seed=int(fx["seed"]), emb_scale=float(fx["emb_scale"]),
                               ln_jitter=float(fx["ln_jitter"]))
    ro, rd = orc.get_rays(fx["pose"], fx["intrinsics"], int(fx["H"]), int(fx["W"]))
    model = orc.OracleNeRF(spec, params)
    keep = {}
    model.run(ro, rd, return_feats=1, keep=keep)
    for st in range(3):
        sig, ds, rb, u01 = model.stage_sigmas(ro, rd, keep[f"bins{st}"], st)
        assert torch.equal(sig, keep[f"sigmas{st}"]), st
        assert torch.equal(orc.composite_weights(rb, sig), keep[f"weights{st}"]), st
        assert torch.equal(orc.composite_from_ds(ds), keep[f"weights{st}"]), st
        assert u01.shape == (ro.shape[0], sig.shape[1], 3) and bool(((u01 >= 0) & (u01 <= 1)).all())


def test_oracle_steps_match_reference_golden():
    u = np.load(os.path.join(GOLDEN, "units.npz"))
    ro, rd = orc.get_rays(u["rays_pose"], u["rays_intr"], 16, 24)
    np.testing.assert_array_equal(ro.numpy(), u["rays_o"])
    np.testing.assert_array_equal(rd.numpy(), u["rays_d"])
    n, f = orc.near_far_from_aabb(torch.from_numpy(u["nf_o"]), torch.from_numpy(u["nf_d"]),
                                  torch.tensor([-128.0] * 3 + [128.0] * 3), 0.2)
    np.testing.assert_array_equal(n.numpy(), u["nf_near"])
    np.testing.assert_array_equal(f.numpy(), u["nf_far"])
    assert (u["nf_near"][:32] == 1e9).all()          # rays that miss the box
    np.testing.assert_array_equal(orc.contract(torch.from_numpy(u["contract_x"])).numpy(),
                                  u["contract_z"])
    for T0, T in [(128, 65), (64, 33)]:
        out, inds = orc.sample_pdf(torch.from_numpy(u[f"pdf{T0}_bins"]),
                                   torch.from_numpy(u[f"pdf{T0}_w"]), T, return_inds=True)
        np.testing.assert_array_equal(out.numpy(), u[f"pdf{T0}_out"])
        np.testing.assert_array_equal(inds.numpy(), u[f"pdf{T0}_inds_oracle"])


# ------------------------------------------------------------------ SH KAT --

def _real_sh_scipy(dirs, degree):
    from scipy.special import sph_harm_y
    x, y, z = dirs.T.astype(np.float64)
    theta = np.arccos(np.clip(z, -1, 1))
    phi = np.arctan2(y, x)
    out = np.zeros((dirs.shape[0], degree * degree))
    for l in range(degree):
        for m in range(0, l + 1):
            Y = sph_harm_y(l, m, theta, phi)
            if m == 0:
                out[:, l * l + l] = Y.real
            else:
                out[:, l * l + l + m] = np.sqrt(2) * Y.real
                out[:, l * l + l - m] = np.sqrt(2) * Y.imag
    return out


@pytest.mark.parametrize("degree", [1, 2, 3, 4, 5, 6, 7, 8])
def test_sh_oracle_known_answer_scipy(oracle_lib, degree):
    rng = np.random.default_rng(degree)
    d = rng.standard_normal((1000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    got = enc.sh_encode_forward(d, degree)
    ref = _real_sh_scipy(d, degree)
    np.testing.assert_allclose(got, ref, atol=2e-6 * 4 ** (degree / 4), rtol=1e-5)


def test_sh_oracle_jacobian_matches_finite_differences(oracle_lib):
    rng = np.random.default_rng(0)
    d = rng.uniform(-1, 1, (200, 3)).astype(np.float64)
    _, jac = enc.sh_encode_forward(d.astype(np.float32), 8, calc_dy_dx=True)
    jac = jac.reshape(200, 3, 64)
    h = 1e-3
    for ax in range(3):
        dp, dm = d.copy(), d.copy()
        dp[:, ax] += h
        dm[:, ax] -= h
        num = (enc.sh_encode_forward(dp.astype(np.float32), 8).astype(np.float64) -
               enc.sh_encode_forward(dm.astype(np.float32), 8).astype(np.float64)) / (2 * h)
        np.testing.assert_allclose(jac[:, ax], num, atol=5e-2, rtol=2e-2)


def test_sh_backward_is_jacobian_transpose(oracle_lib):
    rng = np.random.default_rng(1)
    d = rng.standard_normal((64, 3)).astype(np.float32)
    _, jac = enc.sh_encode_forward(d, 4, calc_dy_dx=True)
    g = rng.standard_normal((64, 16)).astype(np.float32)
    gin = enc.sh_encode_backward(g, d, 4, jac)
    ref = np.einsum("bc,bdc->bd", g.astype(np.float64), jac.reshape(64, 3, 16).astype(np.float64))
    np.testing.assert_allclose(gin, ref, rtol=1e-5, atol=1e-5)


# ---------------------------------------------------------------- grid KAT --

def test_grid_dense_levels_equal_grid_sample(oracle_lib):
    """Dense levels: kernel trilinear == F.grid_sample(border, align_corners=False)."""
    spec = synth.GridSpec(num_levels=3, level_dim=4, log2_hashmap_size=22, desired_resolution=40,
                          base_resolution=10)
    offs = spec.offsets()
    L, C = spec.num_levels, spec.level_dim
    rng = np.random.default_rng(3)
    emb = rng.uniform(-1, 1, (int(offs[-1]), C)).astype(np.float32)
    x = rng.uniform(0, 1, (2000, 3)).astype(np.float32)
    x[:8] = [[0, 0, 0], [1, 1, 1], [0, 1, 0.5], [1e-7, 0.999999, 0.5],
             [0.5, 0.5, 0.5], [0.25, 0.75, 1.0], [1.0, 0.0, 0.0], [0.03125, 0.0625, 0.125]]
    out = enc.grid_encode_forward(x, emb, offs, L, spec.S, spec.base_resolution)
    res = enc.grid_level_resolutions(L, spec.S, spec.base_resolution)
    for l in range(L):
        r = res[l]
        assert r ** 3 <= offs[l + 1] - offs[l], "test needs dense levels"
        vol = torch.from_numpy(emb[offs[l]:offs[l] + r ** 3].astype(np.float64))
        vol = vol.view(r, r, r, C).permute(3, 0, 1, 2)[None]          # [1, C, z, y, x]
        g = torch.from_numpy(2 * x.astype(np.float64) - 1).view(1, 1, 1, -1, 3)
        ref = F.grid_sample(vol, g, mode="bilinear", padding_mode="border", align_corners=False)
        ref = ref.view(C, -1).T.numpy()
        np.testing.assert_allclose(out[l], ref, atol=1e-5, rtol=0)   # fp32 position vs fp64


def test_grid_hash_rows_literal(oracle_lib):
    spec = synth.ModelSpec().grid               # L16 C2 T=2^19, desired 4096
    offs = spec.offsets()
    L = spec.num_levels
    res = enc.grid_level_resolutions(L, spec.S, spec.base_resolution)
    x = np.array([[0.1, 0.2, 0.3], [0.9, 0.5, 0.05], [0.5, 0.5, 0.5]], np.float32)
    emb = np.zeros((int(offs[-1]), 2), np.float32)
    _, rows = enc.grid_encode_forward(x, emb, offs, L, spec.S, spec.base_resolution,
                                      return_rows=True)
    P1, P2, M = 2654435761, 805459861, 0xFFFFFFFF
    for l in (5, 10, 15):
        r, size = res[l], int(offs[l + 1] - offs[l])
        assert r ** 3 > size
        for b in range(3):
            pos = [np.clip(np.float32(np.float32(x[b, d]) * np.float32(r)) - np.float32(0.5), 0, r - 1)
                   for d in range(3)]
            cell = [int(np.floor(p)) for p in pos]
            # corner 0 (no +1): a literal xor-hash of the cell
            h = (cell[0] ^ ((cell[1] * P1) & M) ^ ((cell[2] * P2) & M)) % size
            assert rows[l, b, 0] == h
    assert res[15] == 4096 and res[0] == 16


def test_grid_resolution_table_matches_survey():
    s = synth.ModelSpec().s_grid
    res = enc.grid_level_resolutions(16, s.S, 16)
    assert res[6] == 64 and res[9] == 128 and res[12] == 256 and res[15] == 512
    py = [int(np.ceil(16 * s.per_level_scale ** l)) for l in range(16)]
    assert py[6] == 65 and py[15] == 513                   # storage vs indexing (H4)


def test_grid_backward_is_adjoint_of_forward(oracle_lib):
    spec = synth.GridSpec(5, 2, 12, 256)
    offs = spec.offsets()
    rng = np.random.default_rng(5)
    emb = rng.uniform(-1, 1, (int(offs[-1]), 2)).astype(np.float32)
    x = rng.uniform(-0.05, 1.05, (3000, 3)).astype(np.float32)       # includes OOB points
    out = enc.grid_encode_forward(x, emb, offs, 5, spec.S, 16)
    g = rng.standard_normal(out.shape).astype(np.float32)
    gemb = enc.grid_encode_backward(g, x, emb, offs, 5, spec.S, 16)
    lhs = float((g.astype(np.float64) * out.astype(np.float64)).sum())
    rhs = float((gemb.astype(np.float64) * emb.astype(np.float64)).sum())
    assert abs(lhs - rhs) < 1e-3 * max(1.0, abs(lhs))
    oob = ((x < 0) | (x > 1)).any(1)
    assert oob.any() and (out[:, oob] == 0).all()


def test_grid_input_gradient_matches_finite_differences(oracle_lib):
    spec = synth.GridSpec(4, 2, 14, 64)
    offs = spec.offsets()
    rng = np.random.default_rng(6)
    emb = rng.uniform(-1, 1, (int(offs[-1]), 2)).astype(np.float32)
    x = rng.uniform(0.05, 0.95, (256, 3)).astype(np.float64)
    out, dy = enc.grid_encode_forward(x.astype(np.float32), emb, offs, 4, spec.S, 16,
                                      calc_dy_dx=True)
    dy = dy.reshape(256, 4, 3, 2)
    h = 1e-4
    ok = 0
    for ax in range(3):
        xp, xm = x.copy(), x.copy()
        xp[:, ax] += h
        xm[:, ax] -= h
        fp = enc.grid_encode_forward(xp.astype(np.float32), emb, offs, 4, spec.S, 16)
        fm = enc.grid_encode_forward(xm.astype(np.float32), emb, offs, 4, spec.S, 16)
        num = ((fp.astype(np.float64) - fm) / (2 * h)).transpose(1, 0, 2)      # [B, L, C]
        close = np.isclose(dy[:, :, ax], num, rtol=5e-2, atol=5e-2)
        ok += close.mean()
    assert ok / 3 > 0.97       # a few points straddle a cell boundary within +-h


def test_weight_decay_closed_form(oracle_lib):
    spec = synth.GridSpec(5, 2, 10, 128)
    offs = spec.offsets()
    rng = np.random.default_rng(7)
    emb = rng.standard_normal((int(offs[-1]), 2)).astype(np.float32)
    grad = rng.standard_normal(emb.shape).astype(np.float32)
    got = enc.grad_weight_decay(emb, grad, offs, 0.1, 5)
    exp = grad.copy()
    for l in range(5):
        a, b = offs[l], offs[l + 1]
        exp[a:b] += (np.float32(0.2) * emb[a:b]) / np.float32(b - a)
    np.testing.assert_allclose(got, exp, rtol=1e-6, atol=1e-7)


def test_total_variation_small_case_python_loop(oracle_lib):
    spec = synth.GridSpec(2, 2, 12, 8, base_resolution=4)     # dense 4^3 and 8^3
    offs = spec.offsets()
    rng = np.random.default_rng(8)
    emb = rng.standard_normal((int(offs[-1]), 2)).astype(np.float32)
    x = rng.uniform(0, 1, (50, 3)).astype(np.float32)
    got = enc.grad_total_variation(x, emb, np.zeros_like(emb), offs, 1.0, 2, spec.S, 4)
    exp = np.zeros_like(emb, dtype=np.float64)
    res = enc.grid_level_resolutions(2, spec.S, 4)
    for l in range(2):
        r = res[l]
        for b in range(50):
            cell = [int(np.floor(min(max(x[b, d] * r - 0.5, 0), r - 1))) for d in range(3)]
            idx = lambda c: offs[l] + (c[0] + c[1] * r + c[2] * r * r) % (offs[l + 1] - offs[l])
            here = idx(cell)
            s = np.zeros(2)
            q = np.zeros(2)
            for d in range(3):
                for delta, ok in ((1, cell[d] < r), (-1, cell[d] > 0)):
                    if ok:
                        c2 = list(cell)
                        c2[d] += delta
                        v = emb[here].astype(np.float64) - emb[idx(c2)]
                        s += v
                        q += v * v
            exp[here] += (1.0 / 6) * s / np.sqrt(q + 1e-9)
    np.testing.assert_allclose(got, exp, rtol=1e-4, atol=1e-5)


# -------------------------------------------------------------------- freq --

def test_freq_oracle_closed_form(oracle_lib):
    rng = np.random.default_rng(9)
    x = rng.uniform(-1, 1, (100, 3)).astype(np.float32)
    out = enc.freq_encode_forward(x, 6)
    parts = [x.astype(np.float64)]
    for f in range(6):
        parts += [np.sin(x * 2.0 ** f), np.cos(x * 2.0 ** f)]
    np.testing.assert_allclose(out, np.concatenate(parts, 1), atol=3e-6)
    g = rng.standard_normal(out.shape).astype(np.float32)
    gin = enc.freq_encode_backward(g, out, 6)
    ref = g[:, :3].astype(np.float64)
    for f in range(6):
        s = 3 + 6 * f
        ref = ref + 2.0 ** f * (g[:, s:s + 3] * np.cos(x * 2.0 ** f) - g[:, s + 3:s + 6] * np.sin(x * 2.0 ** f))
    np.testing.assert_allclose(gin, ref, rtol=1e-4, atol=1e-4)


def test_torch_cpu_row_sum_order():
    """The summation order the HIP sample_pdf normaliser reproduces
    (raymarch_device.h torch_row_sum): 8-lane vectors, 4 round-robin
    accumulators, scalar tail first, lanes in sequence -- equal to torch.sum
    on the CPU bit for bit, for every row length on the path."""
    f = np.float32

    def emulate(x):
        n = x.shape[1]
        nv = n // 8
        acc = [np.zeros((x.shape[0], 8), f) for _ in range(4)]
        for v in range(nv):
            acc[v % 4] = (acc[v % 4] + x[:, v * 8:(v + 1) * 8]).astype(f)
        a = acc[0]
        for m in range(1, 4):
            a = (a + acc[m]).astype(f)
        t = np.zeros(x.shape[0], f)
        for k in range(nv * 8, n):
            t = (t + x[:, k]).astype(f)
        for l in range(8):
            t = (t + a[:, l]).astype(f)
        return t

    g = torch.Generator().manual_seed(0)
    for n in (32, 33, 64, 65, 128, 129):
        x = torch.rand(2048, n, generator=g) ** 4 * 3 + 0.01
        assert np.array_equal(emulate(x.numpy()), torch.sum(x, -1).numpy()), n
