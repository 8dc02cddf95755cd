"""Fused ray-march pipeline on the MI355X vs the CPU oracle.

Bar (BASELINE.json north_star): integer results (searchsorted indices, corner
rows) bit-exact on identical float inputs; RGB / depth / feature / sigma
within 1e-3 of the reference (absolute; depth relative, since it is measured
in world units up to ~220).  Goldens come from the reference's own Python
(tests/golden, made by tools/make_golden.py).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from helpers import make_net, max_abs, oracle_for, spec_from_fixture
from oracle import renderer as orc
from oracle import synth

pytestmark = pytest.mark.gpu

TOL = 1e-3


# ----------------------------------------------------------- step kernels --

def test_get_rays_matches_reference(hip_lib, cuda):
    from samnerf_amd import ops
    u = np.load(os.path.join(GOLDEN, "units.npz"))
    ro, rd = ops.get_rays(u["rays_pose"], u["rays_intr"], 16, 24, device=cuda)
    np.testing.assert_array_equal(ro.cpu().numpy(), u["rays_o"])
    np.testing.assert_allclose(rd.cpu().numpy(), u["rays_d"], rtol=0, atol=2e-6)
    pose, intr = synth.gui_camera(512, 512)                     # the GUI camera: exact
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=cuda)
    o2, d2 = orc.get_rays(pose, intr, 512, 512)
    assert torch.equal(rd.cpu(), d2) and torch.equal(ro.cpu(), o2)
    # a row band equals the same rows of the full view (multi-GPU sharding)
    rb, db = ops.get_rays(pose, intr, 512, 512, device=cuda, row0=64, rows=64)
    assert torch.equal(db.cpu(), d2[64 * 512:128 * 512])


def test_near_far_and_contract_bit_exact(hip_lib, cuda):
    from samnerf_amd import ops
    u = np.load(os.path.join(GOLDEN, "units.npz"))
    n, f = ops.near_far(torch.from_numpy(u["nf_o"]).to(cuda), torch.from_numpy(u["nf_d"]).to(cuda),
                        [-128.0] * 3 + [128.0] * 3, 0.2)
    np.testing.assert_array_equal(n.cpu().numpy(), u["nf_near"])
    np.testing.assert_array_equal(f.cpu().numpy(), u["nf_far"])
    z = ops.contract(torch.from_numpy(u["contract_x"]).to(cuda))
    np.testing.assert_array_equal(z.cpu().numpy(), u["contract_z"])


@pytest.mark.parametrize("T0,T", [(128, 65), (64, 33)])
def test_sample_pdf_indices_exact(hip_lib, cuda, T0, T):
    from samnerf_amd import ops
    u = np.load(os.path.join(GOLDEN, "units.npz"))
    bins = torch.from_numpy(u[f"pdf{T0}_bins"]).to(cuda)
    w = torch.from_numpy(u[f"pdf{T0}_w"]).to(cuda)
    out, inds = ops.sample_pdf(bins, w, T, return_inds=True)
    ref_inds = u[f"pdf{T0}_inds_oracle"]
    mism = (inds.cpu().numpy() != ref_inds).mean()
    assert mism == 0.0, f"searchsorted index mismatch rate {mism}"
    np.testing.assert_allclose(out.cpu().numpy(), u[f"pdf{T0}_out"], rtol=0, atol=1e-6)


def test_composite_weights_match_oracle(hip_lib, cuda):
    from samnerf_amd import ops
    g = torch.Generator().manual_seed(3)
    rb = torch.sort(torch.rand(512, 65, generator=g) * 50, -1).values
    rb[0] = 7.0                                              # zero-width bins
    sig = torch.rand(512, 64, generator=g) * 5
    sig[1] = 0.0
    ref = orc.composite_weights(rb, sig)
    got = ops.composite_weights(rb.to(cuda), sig.to(cuda)).cpu()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=2e-6, atol=1e-7)


# ------------------------------------------------------------- fused path --

def _check_outputs(out, ref, H=None, W=None, tol=TOL):
    errs = {}
    errs["image"] = max_abs(out["image"], ref["image"])
    errs["weights_sum"] = max_abs(out["weights_sum"], ref["weights_sum"])
    d_ref = ref["depth"].float()
    errs["depth_rel"] = ((out["depth"].cpu() - d_ref).abs() / d_ref.abs().clamp(min=1.0)).max().item()
    if "samvit" in ref:
        errs["samvit"] = max_abs(out["samvit"].reshape(-1, 256), ref["samvit"].reshape(-1, 256))
    for k, v in errs.items():
        assert v < tol, f"{k}: {v:.3e} >= {tol} (all: {errs})"
    return errs


@pytest.mark.parametrize("head_mode", [0, 1])
@pytest.mark.parametrize("name", ["render_small_rgb", "render_small_sam",
                                  "render_small_sam_default_init", "render_full_sam"])
def test_fused_render_matches_reference_golden(hip_lib, cuda, monkeypatch, name, head_mode):
    """Both precision modes against the reference's own outputs: head_mode 0
    (grid_mlp, SAM head on f16x3 MFMA) and 1 (every GEMM on
    exact fp32 MFMA)."""
    fx = np.load(os.path.join(GOLDEN, name + ".npz"))
    spec = spec_from_fixture(fx)
    params = synth.make_params(spec, seed=int(fx["seed"]), emb_scale=float(fx["emb_scale"]),
                               ln_jitter=float(fx["ln_jitter"]))
    net = make_net(spec, params, cuda)
    net.head_mode = head_mode                        # the fused path's GEMM precision
    ro = torch.from_numpy(fx["rays_o"]).to(cuda)
    rd = torch.from_numpy(fx["rays_d"]).to(cuda)
    H, W = int(fx["H"]), int(fx["W"])
    out = net.render(ro, rd, staged=False, return_feats=1, H=H, W=W)
    ref = {k: torch.from_numpy(fx[k]) for k in ("image", "depth", "weights_sum")}
    if spec.with_sam:
        ref["samvit"] = torch.from_numpy(fx["samvit"])
    errs = _check_outputs(out, ref)
    print(name, head_mode, errs)


def test_fused_equals_unfused_torch_path(hip_lib, cuda):
    """The fused kernels vs the reference's unfused op sequence running on the
    same GPU with the drop-in encoders (the reference-equivalent baseline)."""
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_params(spec, seed=21, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(9))
    from samnerf_amd import ops
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    with torch.no_grad():
        fused = net.run(ro, rd, return_feats=1)
        torch_path = net.run_torch(ro, rd, return_feats=1)
    _check_outputs(fused, {k: v.cpu() for k, v in torch_path.items()})


def test_fused_full_view_parity_on_sampled_rays(hip_lib, cuda):
    """512x512 view (config 3 shape): full render on the GPU, oracle on a
    seeded sample of 192 rays (rays are independent), plus view-wide
    invariants."""
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_params(spec, seed=33, emb_scale=0.5, ln_jitter=0.0)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(512, 512, rot=synth.random_rotation(2))
    from samnerf_amd import ops
    ro, rd = ops.get_rays(pose, intr, 512, 512, device=cuda)
    out = net.render(ro, rd, staged=False, return_feats=1)
    sv = out["samvit"].reshape(-1, 256)
    assert torch.isfinite(out["image"]).all() and torch.isfinite(sv).all()
    ws = out["weights_sum"]
    assert (ws > 0.999).all() and (ws < 1.001).all()          # last_sample background
    idx = torch.from_numpy(np.random.default_rng(0).choice(512 * 512, 192, replace=False))
    ref = oracle_for(spec, params).run(ro[idx.to(cuda)].cpu(), rd[idx.to(cuda)].cpu(), return_feats=1)
    sub = {k: v[idx.to(cuda)] for k, v in out.items() if k != "samvit"}
    sub["samvit"] = sv[idx.to(cuda)]
    errs = _check_outputs(sub, ref)
    print("512x512 sampled", errs)
    # LayerNorm with unit gain / zero bias: every row has mean 0 and variance
    # var(x) / (var(x) + 1e-5) <= 1
    var = sv.var(1, unbiased=False)
    assert sv.mean(1).abs().max() < 1e-4 and var.max() < 1 + 1e-4 and var.median() > 0.9


def test_fused_staged_and_cam_near_far(hip_lib, cuda):
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=11, prop_log2=10)
    params = synth.make_params(spec, seed=4, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    net.opt.max_ray_batch = 1000
    pose, intr = synth.gui_camera(48, 48, rot=synth.random_rotation(4))
    from samnerf_amd import ops
    ro, rd = ops.get_rays(pose, intr, 48, 48, device=cuda)
    a = net.render(ro, rd, staged=False, return_feats=1, H=48, W=48)
    b = net.render(ro, rd, staged=True, return_feats=1, H=48, W=48)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    cnf = torch.tensor([[0.3, 5.0]], device=cuda)
    c = net.render(ro, rd, staged=False, cam_near_far=cnf, return_feats=1)
    ref = oracle_for(spec, params)
    # oracle with the same clamp (renderer.py:234-236) via the torch path on CPU
    r2 = net.run_torch(ro, rd, cam_near_far=cnf.expand(ro.shape[0], 2), return_feats=1)
    _check_outputs(c, {k: v.cpu() for k, v in r2.items()})
    del ref


def test_fused_rgb_only_and_background(hip_lib, cuda):
    fx = np.load(os.path.join(GOLDEN, "render_small_rgb.npz"))
    spec = spec_from_fixture(fx)
    params = synth.make_params(spec, seed=int(fx["seed"]), emb_scale=float(fx["emb_scale"]))
    net = make_net(spec, params, cuda)
    ro = torch.from_numpy(fx["rays_o"]).to(cuda)
    rd = torch.from_numpy(fx["rays_d"]).to(cuda)
    a = net.run(ro, rd, bg_color=0.0)
    ref = oracle_for(spec, params).run(ro.cpu(), rd.cpu(), bg_color=0.0)
    _check_outputs(a, ref)
    assert "samvit" not in a


def _head_errors(net, rows):
    """max |samvit - float64| of the f16x3 head, the exact fp32 MFMA head and
    torch's fp32 CPU head on the same rows."""
    import copy
    from samnerf_amd.fused import FusedRenderer
    f16 = FusedRenderer(net, head_mode=0).sam_head(rows).cpu().double()
    ex = FusedRenderer(net, head_mode=1).sam_head(rows).cpu().double()
    head = copy.deepcopy(net.samvit_mlp).cpu()
    x = rows[:, :163].cpu()
    with torch.no_grad():
        ref = head.double()(x.double())
        c32 = copy.deepcopy(net.samvit_mlp).cpu().float()(x).double()
    e = {k: (v - ref).abs().max().item() for k, v in (("f16x3", f16), ("exact_mfma", ex), ("cpu_fp32", c32))}
    e["f16x3_vs_exact_rel"] = ((f16 - ex).abs().max() / ref.abs().max()).item()
    return e


def test_sam_head_f16x3_is_fp32_equivalent(hip_lib, cuda):
    """The default head (f16x3: three fp16 MFMA products per fp32 product on
    power-of-two scaled operands, csrc/f16x3.h) on identical head-input rows:
    as close to the float64 head as the exact fp32 MFMA head and torch's fp32
    CPU head are (within 2x of the better of the two), and within 1e-6 of the
    exact head relative to the output scale."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    params = synth.make_params(spec, seed=8, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(96, 96, rot=synth.random_rotation(1))
    ro, rd = ops.get_rays(pose, intr, 96, 96, device=cuda)
    rows = torch.empty(96 * 96, 164, device=cuda)
    full = FusedRenderer(net).render(ro, rd, rows=rows)["samvit"]
    e = _head_errors(net, rows)
    print("head vs float64:", e)
    assert e["f16x3"] <= 2.0 * min(e["exact_mfma"], e["cpu_fp32"]) + 1e-7, e
    assert e["f16x3_vs_exact_rel"] < 1e-6, e
    # the render's head is the same kernel on the same rows
    assert torch.equal(full, FusedRenderer(net).sam_head(rows))


def test_sam_head_f16x3_scaling_over_wide_ranges(hip_lib, cuda):
    """Rows whose magnitudes span 1e-30 .. 1e6 (per ray), all-zero rows and a
    single huge entry: the power-of-two operand scaling keeps the f16x3 head
    at fp32-equivalent error (fp16 alone has a 2^-14 .. 65504 normal range)."""
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=11, prop_log2=10)
    params = synth.make_params(spec, seed=5, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    g = torch.Generator().manual_seed(3)
    n = 1000
    rows = torch.randn(n, 164, generator=g)
    rows *= 10.0 ** (torch.rand(n, 1, generator=g) * 36 - 30)     # per-ray scale 1e-30 .. 1e6
    rows[:7] = 0.0                                                 # all-zero rays
    rows[7:20, 162] = 3e5                                          # a huge depth, small rest
    rows[:, 163] = 0.0
    e = _head_errors(net, rows.to(cuda))
    print("wide-range head vs float64:", e)
    assert e["f16x3"] <= 2.0 * min(e["exact_mfma"], e["cpu_fp32"]) + 1e-7, e


@pytest.mark.parametrize("n", [1000, 128 * 300 + 37, 128 * 1024])
def test_sam_head_persistent_form_bit_identical(hip_lib, cuda, n):
    """The persistent 32-ray head (k_sam_head_h16q, the product through round
    5 and the diagnostic build's form 0: one workgroup per CU over 128-ray
    tiles, the next tile's rows streamed into LDS, the weight ring running on
    across tiles) equals the one-block-per-tile kernel (diagnostic form 4) bit
    for bit: ragged tails, more tiles than compute units (several tiles per
    workgroup), rows ending at the allocation's end (clamped row pieces)."""
    from samnerf_amd import _lib
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=11, prop_log2=10)
    params = synth.make_params(spec, seed=6, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    g = torch.Generator().manual_seed(n)
    rows = torch.randn(n, 164, generator=g)
    rows *= 10.0 ** (torch.rand(n, 1, generator=g) * 8 - 4)
    rows[:, 163] = 0.0
    rows = rows.to(cuda)
    out = {}
    try:
        with _lib.diag_library():
            for form in ("0", "4"):
                os.environ["SAMNERF_HEAD_V"] = form
                out[form] = FusedRenderer(net).sam_head(rows)
    finally:
        os.environ.pop("SAMNERF_HEAD_V", None)
    assert torch.isfinite(out["0"]).all()
    assert torch.equal(out["0"], out["4"])



@pytest.mark.parametrize("form", ["30", "31"])
@pytest.mark.parametrize("n", [1000, 128 * 300 + 37, 128 * 1024])
def test_sam_head_w8_form_is_fp32_equivalent(hip_lib, cuda, n, form):
    """The 16-ray two-waves-per-SIMD head (k_sam_head_w8; form 30, the
    product since round 6: one 8-wave workgroup per CU, 128-ray tiles; 31: two
    4-wave workgroups per CU, 64-ray tiles; v_mfma_f32_16x16x32_f16, 32-deep
    k-blocks) on rows spanning 1e-4 .. 1e4 per ray: as close to the float64
    head as the exact fp32 MFMA head (within 2x), within 1e-6 of the 32-ray
    f16x3 head (k_sam_head_h16q, diagnostic form 0) relative to the output
    scale; form 30 of the diagnostic build is the product bit for bit; ragged
    tails and several tiles per workgroup (the rows streamed into LDS, the
    weight ring across tiles)."""
    import copy
    from samnerf_amd import _lib
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=11, prop_log2=10)
    params = synth.make_params(spec, seed=6, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    g = torch.Generator().manual_seed(n)
    rows = torch.randn(n, 164, generator=g)
    rows *= 10.0 ** (torch.rand(n, 1, generator=g) * 8 - 4)
    rows[:5] = 0.0
    rows[:, 163] = 0.0
    rows = rows.to(cuda)
    product = FusedRenderer(net).sam_head(rows).cpu().double()
    ex = FusedRenderer(net, head_mode=1).sam_head(rows).cpu().double()
    try:
        with _lib.diag_library():
            os.environ["SAMNERF_HEAD_V"] = "0"
            prod = FusedRenderer(net).sam_head(rows).cpu().double()
            os.environ["SAMNERF_HEAD_V"] = form
            w8 = FusedRenderer(net).sam_head(rows).cpu().double()
    finally:
        os.environ.pop("SAMNERF_HEAD_V", None)
    if form == "30":
        assert torch.equal(w8, product)
    head = copy.deepcopy(net.samvit_mlp).cpu()
    with torch.no_grad():
        ref = head.double()(rows[:, :163].cpu().double())
    assert torch.isfinite(w8).all()
    e_w8 = (w8 - ref).abs().max().item()
    e_ex = (ex - ref).abs().max().item()
    rel = ((w8 - prod).abs().max() / ref.abs().max()).item()
    print("w8 head vs float64", e_w8, "exact", e_ex, "vs product rel", rel)
    assert e_w8 <= 2.0 * e_ex + 1e-7, (e_w8, e_ex)
    assert rel < 1e-6, rel

def test_exact_fp32_mode_vs_oracle(hip_lib, cuda):
    """head_mode 1 runs grid_mlp on v_mfma_f32_32x32x2_f32 (an fma chain per
    k pair) as well as the SAM head: against the oracle (torch CPU GEMMs in
    another summation order) it sits at fp32 rounding, and the default f16x3
    mode agrees with it at that level (both fp32-equivalent)."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_params(spec, seed=12, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(3))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    exact = FusedRenderer(net, head_mode=1).render(ro, rd)
    fast = FusedRenderer(net, head_mode=0).render(ro, rd)
    ref = oracle_for(spec, params).run(ro.cpu(), rd.cpu(), return_feats=1)
    e = {k: max_abs(exact[k], ref[k]) for k in ("image", "weights_sum", "samvit")}
    f = {k: max_abs(fast[k], ref[k]) for k in ("image", "weights_sum", "samvit")}
    print("exact vs oracle", e, "f16x3 vs oracle", f, "f16x3 vs exact",
          max_abs(exact["samvit"], fast["samvit"]))
    assert e["image"] < 2e-6 and e["weights_sum"] < 2e-6 and e["samvit"] < 2e-5, e
    assert f["image"] < 2e-6 and f["weights_sum"] < 2e-6 and f["samvit"] < 2e-5, f
    assert max_abs(exact["samvit"], fast["samvit"]) < 2e-5


@pytest.mark.parametrize("small", ["hashed", "dense"])
def test_final_joint_scale_over_wide_level_ranges(hip_lib, cuda, small):
    """k_final's layer 1 takes ONE f16x3 scale over both k-blocks
    (all 16 levels, SAMNERF_FINAL_JOINT), so a level far below the column's
    max keeps fewer bits in its fp16 halves.  With the hashed (or the dense)
    levels' embeddings 2^-20 of the others, the default form still sits at
    fp32 rounding against the oracle and the exact-fp32 form, as at equal
    magnitudes (test_exact_fp32_mode_vs_oracle)."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True)
    params = dict(synth.make_params(spec, seed=13, emb_scale=0.5, ln_jitter=0.1))
    net = make_net(spec, params, cuda)
    off5 = int(net.grid.offsets[5])                           # levels 0-4 dense, 5-15 hashed
    emb = np.array(params["grid.embeddings"], dtype=np.float32, copy=True)
    if small == "hashed":
        emb[off5:] *= np.float32(2.0 ** -20)
    else:
        emb[:off5] *= np.float32(2.0 ** -20)
    params["grid.embeddings"] = emb
    with torch.no_grad():
        net.grid.embeddings.copy_(torch.from_numpy(emb))
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(8))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    exact = FusedRenderer(net, head_mode=1).render(ro, rd)
    fast = FusedRenderer(net, head_mode=0).render(ro, rd)
    ref = oracle_for(spec, params).run(ro.cpu(), rd.cpu(), return_feats=1)
    e = {k: max_abs(exact[k], ref[k]) for k in ("image", "weights_sum", "samvit")}
    f = {k: max_abs(fast[k], ref[k]) for k in ("image", "weights_sum", "samvit")}
    print(small, "exact vs oracle", e, "f16x3 vs oracle", f)
    assert e["image"] < 2e-6 and e["weights_sum"] < 2e-6 and e["samvit"] < 2e-5, e
    assert f["image"] < 2e-6 and f["weights_sum"] < 2e-6 and f["samvit"] < 2e-5, f
    assert max_abs(exact["samvit"], fast["samvit"]) < 2e-5


@pytest.mark.parametrize("mode", ["ref", "box4"])
def test_gather_variants_bit_identical(hip_lib, cuda, monkeypatch, mode, diag):
    """The packed-FMA gathers (default), the per-corner scalar form (ref) and
    the LDS box gathers of k_sgrid_box4 (box4) read the same rows with the same
    weights in the same FMA order: every output bit must agree, including
    for scattered rays (boxes too big for LDS -> direct gathers) and a NaN
    ray (its lanes fall outside the box -> per-lane direct gathers)."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, ROW
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_params(spec, seed=21, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(512, 96, rot=synth.random_rotation(5))
    ro, rd = ops.get_rays(pose, intr, 96, 512, device=cuda)               # 49152 rays
    perm = torch.randperm(ro.shape[0], generator=torch.Generator().manual_seed(0)).to(cuda)
    ro = torch.cat([ro, ro[perm[:8192]]]).contiguous()
    rd = torch.cat([rd, rd[perm[:8192]]]).contiguous()
    rd[-5] = float("nan")
    fr = FusedRenderer(net)
    outs = {}
    for m in ("packed", mode):
        monkeypatch.setenv("SAMNERF_LOOKUP", m)
        rows = torch.empty(ro.shape[0], ROW, device=cuda)
        o = fr.render(ro, rd, rows=rows)
        o["rows"] = rows
        outs[m] = o
    for k in outs["packed"]:
        a = torch.nan_to_num(outs["packed"][k], nan=7.0)
        b = torch.nan_to_num(outs[mode][k], nan=7.0)
        assert torch.equal(a, b), (k, (a - b).abs().max().item())


@pytest.mark.parametrize("head_mode", [0, 1])
def test_ray_segment_paths_agree(hip_lib, cuda, head_mode):
    """k_final spreads each ray's samples over S = 1, 2 or 4 interleaved slots
    by N (more waves for one rank's small share of a view), exchanging optical
    depths by shuffle: the same rays rendered at N >= 65536 (S = 1), 32768 <=
    N < 65536 (S = 2) and N < 32768 (S = 4) must agree to fp32 rounding, and
    the per-sample weights handed to the s_grid gather must too (f_sam
    rows)."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, ROW
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_params(spec, seed=21, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(512, 160, rot=synth.random_rotation(5))
    ro, rd = ops.get_rays(pose, intr, 160, 512, device=cuda)          # 81920 rays
    fr = FusedRenderer(net, head_mode=head_mode)
    outs = {}
    for n in (81920, 40000, 9000):
        rows = torch.empty(n, ROW, device=cuda)
        o = fr.render(ro[:n], rd[:n], rows=rows)
        o["rows"] = rows
        outs[n] = o
    for n in (40000, 9000):
        for k in ("image", "depth", "weights_sum", "samvit", "rows"):
            a, b = outs[81920][k][:n], outs[n][k]
            tol = 1e-4 * (1 + a.abs().max().item()) if k in ("depth", "rows") else 1e-4
            err = (a - b).abs().max().item()
            assert err < tol, (n, k, err)


def test_sam_feature_handoff_stays_on_device(hip_lib, cuda):
    """the fused render's 64x64 feature map goes to the SAM
    decoder interface without leaving the device (nerf/gui.py:143-161 loop)."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    from samnerf_amd.sam_bridge import prepare_sam_features, render_and_predict
    from test_sam_bridge import Recorder
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=11, prop_log2=10)
    net = make_net(spec, synth.make_params(spec, seed=4, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(64, 64)
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    rec = Recorder()
    (masks, orig, low), out = render_and_predict(FusedRenderer(net), rec, ro, rd, 64, 64, 512, 512,
                                                 point_coords=[[256, 256]])
    assert rec.features.is_cuda and rec.coords.is_cuda
    assert torch.equal(rec.features, prepare_sam_features(out["samvit"].view(64, 64, 256)))
    assert orig.tolist() == [[256, 256]] and masks.shape == (1, 512, 512)


def test_render_without_features_matches(hip_lib, cuda):
    """return_feats=0 skips the s_grid composite and the head (the reference
    computes and drops them); the RGB outputs are the same bits."""
    from samnerf_amd import ops
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    net = make_net(spec, synth.make_params(spec, seed=31, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(12))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    a = net.render(ro, rd, return_feats=1)
    b = net.render(ro, rd, return_feats=0)
    assert "samvit" in a and "samvit" not in b
    for k in ("image", "depth", "weights_sum"):
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("n", [0, 1, 63, 65, 257])
def test_fused_ragged_ray_counts(hip_lib, cuda, n):
    """Ray counts that do not fill a wave / block (partial waves in every
    kernel, the S = 4 segment form): outputs match the oracle; N = 0 is a
    no-op returning empty tensors."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True, grid_log2=12, s_grid_log2=11, prop_log2=10)
    params = synth.make_params(spec, seed=14, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(32, 32, rot=synth.random_rotation(13))
    ro, rd = ops.get_rays(pose, intr, 32, 32, device=cuda)
    idx = torch.randperm(1024, generator=torch.Generator().manual_seed(n))[:n].to(cuda)
    out = FusedRenderer(net).render(ro[idx], rd[idx])
    assert out["image"].shape == (n, 3) and out["samvit"].shape == (n, 256)
    if n == 0:
        return
    ref = oracle_for(spec, params).run(ro[idx].cpu(), rd[idx].cpu(), return_feats=1)
    _check_outputs(out, ref)


@pytest.mark.parametrize("n", [70000, 40000, 9000])
def test_final_slot_classes_bit_identical(hip_lib, cuda, monkeypatch, n, diag):
    """k_final's wave-uniform slot paths -- one 16-B load per x-adjacent corner
    pair on dense levels (with the top-cell weight swap) and select-free
    hashed rows -- against the lane-varying form (SAMNERF_FINAL_CLASSES=0),
    and the compile-time layout of the reference grid (LAY 1, the product's
    form) against the same classes taken at run time (SAMNERF_FINAL_LAY=0):
    identical bits, on a view whose far samples reach the top cells of the
    coarse levels, at S = 1 / 2 / 4 segments (n = 70000 / 40000 / 9000)."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, ROW, last_forms
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=29, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(512, 160, rot=synth.random_rotation(17))
    ro, rd = ops.get_rays(pose, intr, 160, 512, device=cuda)
    fr = FusedRenderer(net)
    outs = []
    for cl, lay in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("SAMNERF_FINAL_CLASSES", cl)
        monkeypatch.setenv("SAMNERF_FINAL_LAY", lay)
        rows = torch.empty(n, ROW, device=cuda)
        o = fr.render(ro[:n], rd[:n], rows=rows)
        assert last_forms()[2] == int(lay)          # the form under test is the one that ran
        o["rows"] = rows
        outs.append(o)
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
        assert torch.equal(outs[0][k], outs[2][k]), k


@pytest.mark.parametrize("n", [70000, 9000])
def test_prop_level_classes_bit_identical(hip_lib, cuda, monkeypatch, n, diag):
    """k_prop_sigma with the reference proposal grids' level classes as
    compile-time constants (DDDHH / DDHHH: the 5 levels' loads issued
    together; a dense level whose cell is wave-uniform read through the
    scalar cache) against the run-time form (SAMNERF_PROP_LAY=0: one level's
    loads at a time): every output and the proposal stages' tapped optical
    depths, weights, bins and searchsorted indices, bit for bit."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, ROW, last_forms
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=41, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(512, 160, rot=synth.random_rotation(19))
    ro, rd = ops.get_rays(pose, intr, 160, 512, device=cuda)
    fr = FusedRenderer(net)
    outs = []
    for lay in ("0", "1"):
        monkeypatch.setenv("SAMNERF_PROP_LAY", lay)
        rows = torch.empty(n, ROW, device=cuda)
        o = fr.render(ro[:n], rd[:n], rows=rows, taps=True)
        # the form under test is the one that ran (round 5 found the
        # specialisation unreachable from the render path)
        assert last_forms()[:2] == ([0x1807, 0x1C03] if lay == "1" else [0, 0])
        o["rows"] = rows
        outs.append({k: v.cpu() for k, v in o.items()})
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


def test_fused_render_from_reference_layout_checkpoint(hip_lib, cuda, tmp_path):
    """SURVEY 8f-1 on the device: a model-only checkpoint in the reference's
    layout (utils.py:2046-2074; save_checkpoint writes {epoch, global_step,
    stats, model}) of the golden scene's weights, loaded (weights_only=True)
    into a CUDA network that has already rendered with other weights, renders
    the reference's golden view through the fused kernels; the EMA shadow
    (utils.py:1684-1686) is honoured the same way."""
    from samnerf_amd import checkpoint as ck
    fx = np.load(os.path.join(GOLDEN, "render_small_sam.npz"))
    spec = spec_from_fixture(fx)
    params = synth.make_params(spec, seed=int(fx["seed"]), emb_scale=float(fx["emb_scale"]),
                               ln_jitter=float(fx["ln_jitter"]))
    src = make_net(spec, params, "cpu")
    path = tmp_path / "ngp_ep0003.pth"
    ck.save_checkpoint(src, path, epoch=3, global_step=300)
    other = synth.make_params(spec, seed=int(fx["seed"]) + 1, emb_scale=0.5, ln_jitter=0.2)
    net = make_net(spec, other, cuda)
    ro = torch.from_numpy(fx["rays_o"]).to(cuda)
    rd = torch.from_numpy(fx["rays_d"]).to(cuda)
    H, W = int(fx["H"]), int(fx["W"])
    ref = {k: torch.from_numpy(fx[k]) for k in ("image", "depth", "weights_sum", "samvit")}
    before = net.render(ro, rd, staged=False, return_feats=1, H=H, W=W)
    assert max_abs(before["samvit"].reshape(-1, 256), ref["samvit"].reshape(-1, 256)) > 1e-2
    info = ck.load_checkpoint(net, ck.latest_checkpoint(tmp_path), map_location=cuda)
    assert info["epoch"] == 3 and info["missing"] == [] and info["unexpected"] == []
    out = net.render(ro, rd, staged=False, return_feats=1, H=H, W=W)
    _check_outputs(out, ref)
    # the EMA shadow replaces the weights it covers
    ck.save_checkpoint(make_net(spec, other, "cpu"), tmp_path / "ngp_ep0004.pth", epoch=4,
                       ema_shadow=[p.detach().clone() for p in src.parameters()])
    ck.load_checkpoint(net, str(tmp_path / "ngp_ep0004.pth"), use_ema=True, map_location=cuda)
    _check_outputs(net.render(ro, rd, staged=False, return_feats=1, H=H, W=W), ref)


@pytest.mark.parametrize("surface", [False, True])
def test_ray_tiling_bit_identical(hip_lib, cuda, surface):
    """samnerf_model.view_width (8 x 4 pixel tiles per wave) only changes which
    rays share a wave: every output, the head-input rows included, equals the
    row-major render bit for bit; a width the tiling cannot use (N not a
    multiple of 4 rows) falls back to row-major order."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True)
    params = (synth.make_surface_params(spec, seed=3) if surface
              else synth.make_params(spec, seed=21, emb_scale=0.5, ln_jitter=0.1))
    net = make_net(spec, params, cuda)
    H, W = 96, 128
    pose, intr = synth.gui_camera(W, H, rot=synth.random_rotation(4))
    ro, rd = ops.get_rays(pose, intr, H, W, device=cuda)
    fr = FusedRenderer(net)
    outs = []
    for vw, n in ((0, H * W), (W, H * W), (W, H * W - 2 * W)):
        rows = torch.empty(n, 164, device=cuda)
        o = fr.render(ro[:n], rd[:n], rows=rows, view_width=vw)
        o["rows"] = rows
        outs.append({k: v.cpu() for k, v in o.items()})
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
        assert torch.equal(outs[0][k][:H * W - 2 * W], outs[2][k]), k


def test_fused_proposal_kernel_bit_identical(hip_lib, cuda, monkeypatch, diag):
    """k_prop_fused (ds kept in LDS, one kernel per proposal stage; the
    SAMNERF_PROP_FUSED=1 variant, measured slower) against the default
    two-kernel form k_prop_sigma + k_prop_pdf: every output, head rows
    included, bit for bit, at a full-view-like and a ragged ray count."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=31, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(256, 256, rot=synth.random_rotation(3))
    ro, rd = ops.get_rays(pose, intr, 256, 256, device=cuda)
    fr = FusedRenderer(net)
    for n in (256 * 256, 9001):
        outs = []
        for flag in ("1", "0"):
            monkeypatch.setenv("SAMNERF_PROP_FUSED", flag)
            rows = torch.empty(n, 164, device=cuda)
            o = fr.render(ro[:n], rd[:n], rows=rows)
            o["rows"] = rows
            outs.append({k: v.cpu() for k, v in o.items()})
        for k in outs[0]:
            assert torch.equal(outs[0][k], outs[1][k]), (n, k)


def _twice_equal(render, times=2):
    a = {k: v.cpu() for k, v in render().items()}
    for _ in range(times - 1):
        b = {k: v.cpu() for k, v in render().items()}
        for k in a:
            assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("seg", ["1", "2", "4"])
@pytest.mark.parametrize("head_mode", [0, 1])
def test_final_forms_deterministic(hip_lib, cuda, seg, head_mode):
    """Every k_final form renders the same bits three times in a FRESHLY
    SPAWNED process (tests/final_forms_child.py: the removed round-4 prefetch
    form differed on the first render of a process, so the first render must
    be one of those compared), and the child's digest equals this process's:
    S = 1 / 2 / 4, both precisions, feature rows on, the bench's ray tiling."""
    import subprocess
    import sys
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "final_forms_child.py")
    r = subprocess.run([sys.executable, child, seg, str(head_mode)], capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    digests = [ln.split()[1] for ln in r.stdout.splitlines() if ln.startswith("digest")]
    assert len(digests) == 3 and len(set(digests)) == 1, r.stdout
    from final_forms_child import render_digest
    assert render_digest(seg, head_mode, cuda) == digests[0]


@pytest.mark.parametrize("form", ["exit", "mask_default", "sum_after", "adaptive_density", "adaptive_rgb"])
def test_final_mode_forms_deterministic(hip_lib, cuda, form):
    """The EXIT (N1), GEO (+ k_mask_head), SA and AD instantiations of k_final
    (and the mask kernels after them) render the same bits twice."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    kw, mask, t = {}, False, 0.0
    if form == "exit":
        spec = synth.ModelSpec(with_sam=True)
        params = synth.make_surface_params(spec, seed=3)
        t = 1e-3
    else:
        kw = {"mask_default": dict(mask_type="default"),
              "sum_after": dict(mask_type="default", sum_after_mlp=True),
              "adaptive_density": dict(mask_type="adaptive", adaptive_type="density"),
              "adaptive_rgb": dict(mask_type="adaptive", adaptive_type="rgb", sum_after_mlp=True)}[form]
        spec = synth.ModelSpec(with_sam=False, with_mask=True, **kw)
        params = synth.make_params(spec, seed=17, emb_scale=0.5)
        mask = True
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(256, 128, rot=synth.random_rotation(2))
    ro, rd = ops.get_rays(pose, intr, 128, 256, device=cuda)
    fr = FusedRenderer(net, t_thresh=t)
    _twice_equal(lambda: fr.render(ro, rd, mask=mask, view_width=256))


def test_product_runs_the_specialised_forms(hip_lib, cuda):
    """The product library, on the headline configuration's grids (cfg 3:
    proposal grids DDDHH / DDHHH, power-of-two grid scale, the reference's
    16-level grid), launches the compile-time forms: k_prop_sigma with the
    level classes as constants and k_final's LAY 1 -- at S = 1 and S = 2."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer, last_forms
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=7), cuda)
    pose, intr = synth.gui_camera(512, 160, rot=synth.random_rotation(3))
    ro, rd = ops.get_rays(pose, intr, 160, 512, device=cuda)
    fr = FusedRenderer(net)
    for n in (81920, 40000):
        fr.render(ro[:n], rd[:n])
        assert last_forms() == [0x1807, 0x1C03, 1, 0], n


def test_packed_weight_reuse(hip_lib, cuda):
    """samnerf_model.reuse_packed (round 6): a render on the same per-stream
    workspace with unchanged grid_mlp / SAM-head weights skips the packing
    launches and gives the same bits; an in-place weight update (torch op,
    FusedAdam), a render without features before one with them, and
    head_mode all force a repack -- each render equal, bit for bit, to a fresh
    renderer's."""
    from samnerf_amd import ops
    from samnerf_amd._lib import lib
    from samnerf_amd.fused import FusedRenderer
    from samnerf_amd.optim import FusedAdam
    if lib().samnerf_diag_variants():
        pytest.skip("the diagnostic library always packs")
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    net = make_net(spec, synth.make_params(spec, seed=41, emb_scale=0.5, ln_jitter=0.1), cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(5))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    keys = ("image", "depth", "weights_sum", "samvit")

    def same(a, b):
        return all(torch.equal(a[k], b[k]) for k in keys if k in a or k in b)

    fr = FusedRenderer(net)
    a = fr.render(ro, rd)
    assert fr.last_reuse_packed == 0
    b = fr.render(ro, rd)
    assert fr.last_reuse_packed == 1 and same(a, b)
    with torch.no_grad():                                   # in place: version counter bumps
        net.grid_mlp.net[1].weight.mul_(1.5)
    c = fr.render(ro, rd)
    assert fr.last_reuse_packed == 0 and same(c, FusedRenderer(net).render(ro, rd)) and not same(a, c)
    w = net.samvit_mlp[0].net[2].weight
    w.grad = torch.randn_like(w)
    FusedAdam([w], lr=1e-2).step()                          # raw-pointer update, version bumped
    d = fr.render(ro, rd)
    assert fr.last_reuse_packed == 0 and same(d, FusedRenderer(net).render(ro, rd)) and not same(c, d)
    # another ray count on the same workspace: the packed weights sit at
    # N-independent offsets (raymarch.hip carve())
    n2 = 1000
    h = fr.render(ro[:n2], rd[:n2])
    assert fr.last_reuse_packed == 1 and same(h, FusedRenderer(net).render(ro[:n2], rd[:n2]))
    fr2 = FusedRenderer(net)
    fr2.render(ro, rd, feats=False)                         # the head's weights not packed
    e = fr2.render(ro, rd)
    assert fr2.last_reuse_packed == 0 and same(e, d)
    f = fr2.render(ro, rd)
    assert fr2.last_reuse_packed == 1 and same(f, d)
    fr2._head_mode = 1                                      # (the model struct is rebuilt)
    g = fr2.render(ro, rd)
    assert fr2.last_reuse_packed == 0 and same(g, FusedRenderer(net, head_mode=1).render(ro, rd))
