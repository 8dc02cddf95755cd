"""Whole-view parity of the fused path at BASELINE configs 2 and 3.

Every ray of a 512x512 view with parity weights (embeddings ~U(-0.5, 0.5),
SURVEY.md 8c), not a sample, for an RGB-only model (config 2,
nerf/renderer.py:221-362 without the SAM branch) and a with_sam model (config
3, + renderer.py:364-390):

* the proposal stages' searchsorted indices and resampled bins (sample_pdf,
  nerf/renderer.py:84-119, called at :274-275) bit-exact against the oracle's
  sample_pdf fed the fused kernels' own stage inputs -- the composited
  weights, read through the parity taps (samnerf_set_taps).  This is the
  north star's integer contract on identical float inputs, for k_prop_pdf,
  the kernel the product runs (torch-ordered row sum, double cumsum, quarter
  merge walks);
* those weights against the oracle's compositing (renderer.py:310-326) of the
  same optical depths (fp32, another libm's exp);
* image / depth / weights_sum / samvit of all 262,144 rays within 1e-3 of the
  oracle's full render, with the end-to-end index mismatch rate reported: there
  the two sides' float chains are independent (the proposal MLPs sum in
  another order than torch's CPU GEMM, exp is another libm), so an index can
  flip where u_j lies within an ulp of a cdf entry;
* per sample, every sample of every ray, all three stages: sigma
  (network.py:221-259) against the oracle's density at the fused path's own
  sample positions (its bins, read through the taps) -- the proposal stages'
  delta * sigma, the final stage's sigma itself -- within 1e-3 relative (the
  north star's sigma bar); the final positions bit-exact; the final weights
  against the oracle's compositing (renderer.py:310-326) of the ORACLE's sigma;
* the corner rows (gridencoder.cu:61-79) of every level and corner of every
  final sample of a subset of rays (every 61st), for the main grid (k_final)
  and the s_grid composite (k_sgrid_box4), bit-exact against the oracle's
  get_grid_index restatement (oracle/encoders_oracle.c corner_row).
"""
import numpy as np
import pytest
import torch

from helpers import make_net, oracle_for
from oracle import renderer as orc
from oracle import synth

pytestmark = pytest.mark.gpu

H = W = 512
N = H * W
CHUNK = 16384              # renderer.py:195 max_ray_batch
TOL = 1e-3


@pytest.fixture(scope="module", params=["cfg3_sam", "cfg2_rgb"])
def view(request, hip_lib, cuda):
    """One parity-weight 512x512 view rendered by the product path, taps on."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    with_sam = request.param == "cfg3_sam"
    spec = synth.ModelSpec(with_sam=with_sam)
    params = synth.make_params(spec, seed=33 if with_sam else 34, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(W, H, rot=synth.random_rotation(2 if with_sam else 3))
    ro, rd = ops.get_rays(pose, intr, H, W, device=cuda)
    # tiled, as the bench renders (view_width = W: 8 x 4 pixel tiles per wave);
    # the taps come back in ray order (fused.ray_of_slots)
    out = FusedRenderer(net).render(ro, rd, taps=True, view_width=W)
    torch.cuda.synchronize()
    assert ("samvit" in out) == with_sam
    return {"spec": spec, "params": params, "ro": ro.cpu(), "rd": rd.cpu(), "with_sam": with_sam,
            "out": {k: v.cpu().contiguous() for k, v in out.items()}}


def test_torch_cpu_sum_order_on_this_host():
    """The pdf normaliser's order (raymarch_device.h torch_row_sum) is torch's
    CPU sum order; the comparisons below run torch on this host's CPU."""
    from test_oracle import test_torch_cpu_row_sum_order
    test_torch_cpu_row_sum_order()


def test_composited_weights_match_oracle(view):
    o = view["out"]
    for st in (0, 1):
        ref = orc.composite_from_ds(o[f"ds{st}"])
        got = o[f"w{st}"]
        err = (got - ref).abs().max().item()
        same = (got == ref).float().mean().item()
        print(f"stage {st}: weights max |err| {err:.2e}, identical {same:.4%}")
        assert err < 1e-6, (st, err)


@pytest.mark.parametrize("stage", [0, 1])
def test_prop_indices_bit_exact_full_view(view, stage):
    """searchsorted(cdf, u, right=True) of every ray and resampled bin, both
    proposal stages: identical to the oracle on the fused path's own weights
    and bins (mismatch rate 0)."""
    o = view["out"]
    if stage == 0:
        bins = torch.linspace(0, 1, 129).unsqueeze(0).expand(N, -1)
        w, T, gb, gi = o["w0"], 65, o["bins1"], o["inds1"]
    else:
        bins, w, T, gb, gi = o["bins1"], o["w1"], 33, o["bins2"], o["inds2"]
    ref_b, ref_i = orc.sample_pdf(bins, w, T, return_inds=True)
    mism = (gi.long() != ref_i).sum().item()
    print(f"stage {stage}: {mism} of {ref_i.numel()} indices differ")
    assert mism == 0
    assert torch.equal(gb, ref_b)


def test_every_ray_matches_oracle_render(view):
    """All 262,144 rays vs the oracle's staged render (chunks of 16384 as
    renderer.py:195), plus the end-to-end index mismatch rate."""
    o, model = view["out"], oracle_for(view["spec"], view["params"])
    feats = int(view["with_sam"])
    errs = {"image": 0.0, "weights_sum": 0.0, "depth_rel": 0.0}
    if feats:
        errs["samvit"] = 0.0
    flips = [0, 0]
    n_idx = [0, 0]
    for h in range(0, N, CHUNK):
        keep = {}
        ref = model.run(view["ro"][h:h + CHUNK], view["rd"][h:h + CHUNK], return_feats=feats, keep=keep)
        sl = slice(h, h + CHUNK)
        errs["image"] = max(errs["image"], (o["image"][sl] - ref["image"]).abs().max().item())
        errs["weights_sum"] = max(errs["weights_sum"],
                                  (o["weights_sum"][sl] - ref["weights_sum"]).abs().max().item())
        d = ref["depth"]
        errs["depth_rel"] = max(errs["depth_rel"],
                                ((o["depth"][sl] - d).abs() / d.abs().clamp(min=1.0)).max().item())
        if feats:
            errs["samvit"] = max(errs["samvit"], (o["samvit"][sl] - ref["samvit"]).abs().max().item())
        for st, (T, key) in enumerate(((65, "inds1"), (33, "inds2"))):
            _, ri = orc.sample_pdf(keep[f"bins{st}"], keep[f"weights{st}"], T, return_inds=True)
            flips[st] += (o[key][sl].long() != ri).sum().item()
            n_idx[st] += ri.numel()
    rates = [f / n for f, n in zip(flips, n_idx)]
    print(f"512x512 all rays ({'cfg3' if feats else 'cfg2'}):", errs, "end-to-end index mismatch rates", rates)
    for k, v in errs.items():
        assert v < TOL, (k, v, errs)
    assert max(rates) < 1e-4, rates


def test_view_invariants(view):
    o = view["out"]
    assert torch.isfinite(o["image"]).all()
    if view["with_sam"]:
        assert torch.isfinite(o["samvit"]).all() and o["samvit"].shape == (N, 256)
    assert ((o["weights_sum"] > 0.999) & (o["weights_sum"] < 1.001)).all()   # last_sample bg
    # resampled bins are sorted per ray and span [0, 1]
    for k in ("bins1", "bins2"):
        b = o[k]
        assert (b[:, 1:] >= b[:, :-1]).all() and (b >= 0).all() and (b <= 1).all(), k
    assert int(o["inds1"].min()) >= 1 and int(o["inds1"].max()) <= 129
    assert int(o["inds2"].min()) >= 1 and int(o["inds2"].max()) <= 65
    np.testing.assert_array_equal(o["image"].shape, (N, 3))


SIG_TOL = 1e-3             # north star: sigma within 1e-3 (relative here)


def _rel_err(got, ref):
    """max |got - ref| / |ref| over ref != 0; exact where ref == 0."""
    nz = ref != 0
    assert torch.equal(got[~nz], ref[~nz]), "sigma differs where the oracle's is 0"
    return ((got[nz] - ref[nz]).abs() / ref[nz].abs()).max().item() if nz.any() else 0.0


def test_sigma_every_sample_matches_oracle(view):
    """sigma of every sample of all three stages against the oracle's density
    at the fused path's own positions (OracleNeRF.stage_sigmas, pinned to the
    goldens by tests/test_oracle.py::test_stage_sigmas_restates_run)."""
    o, model = view["out"], oracle_for(view["spec"], view["params"])
    errs = {"ds0_rel": 0.0, "ds1_rel": 0.0, "sigma2_rel": 0.0, "w2_abs": 0.0}
    u2_same = 0
    for h in range(0, N, CHUNK):
        sl = slice(h, h + CHUNK)
        ro, rd = view["ro"][sl], view["rd"][sl]
        n = ro.shape[0]
        bins0 = torch.linspace(0, 1, 129).unsqueeze(0).expand(n, -1)
        for st, bins, key in ((0, bins0, "ds0"), (1, o["bins1"][sl], "ds1")):
            _, ds, _, _ = model.stage_sigmas(ro, rd, bins, st)
            errs[f"{key}_rel"] = max(errs[f"{key}_rel"], _rel_err(o[key][sl], ds))
        sig, _, rb, u01 = model.stage_sigmas(ro, rd, o["bins2"][sl], 2)
        errs["sigma2_rel"] = max(errs["sigma2_rel"], _rel_err(o["sigma2"][sl], sig))
        w_ref = orc.composite_weights(rb, sig)                # the ORACLE's sigma composited
        errs["w2_abs"] = max(errs["w2_abs"], (o["w2"][sl] - w_ref).abs().max().item())
        u2_same += int(torch.equal(o["u2"][sl], u01))
    print(f"512x512 per-sample ({'cfg3' if view['with_sam'] else 'cfg2'}):", errs,
          f"final positions bit-exact in {u2_same} of {N // CHUNK} chunks")
    assert u2_same == N // CHUNK
    for k in ("ds0_rel", "ds1_rel", "sigma2_rel"):
        assert errs[k] < SIG_TOL, (k, errs)
    assert errs["w2_abs"] < 1e-4, errs


def _check_rows(got, pos, grid, what):
    """got [n, 32, 16, 8] int32 (-1 = sample skipped), pos [n, 32, 3]:
    against the oracle's corner rows.  k_final's dense pair loads read the
    top x cell as the pair (top - 1, top) with weights (0, 1) where the
    reference reads (top, top) with (1, 0): same sum bit for bit
    (samnerf_common.h lookup_dense_c2_paired), recorded as such by the tap."""
    from oracle import encoders as enc
    n = got.shape[0]
    _, ref = enc.grid_encode_forward(pos.reshape(-1, 3).numpy(), grid.embeddings, grid.offsets,
                                     grid.L, grid.S, grid.H, return_rows=True)
    ref = torch.from_numpy(ref.astype(np.int64)).reshape(grid.L, n, 32, 8).permute(1, 2, 0, 3)
    g = got.long()
    written = g[..., 0] >= 0
    frac = written.float().mean().item()
    eq = (g == ref).all(-1)
    # dense top-x-cell pairs: corners (2p, 2p + 1) read (R - 1, R) where the
    # reference reads (R, R)
    e, o_ = g[..., 0::2], g[..., 1::2]
    re, ro_ = ref[..., 0::2], ref[..., 1::2]
    edge = ((e == re) & (o_ == ro_)) | ((e == re - 1) & (o_ == re) & (ro_ == re))
    eq_edge = edge.all(-1)
    n_edge = int((eq_edge & ~eq & written).sum())
    bad = int((written & ~eq_edge).sum())
    print(f"{what}: {int(written.sum())} (sample, level) entries written ({frac:.4%}), "
          f"{bad} differ, {n_edge} top-cell pairs")
    assert bad == 0
    return frac


def test_corner_rows_bit_exact(view):
    """k_final's and k_sgrid_box4's corner rows of every level, for the final
    samples of every 61st ray, against the oracle's get_grid_index."""
    o, model = view["out"], oracle_for(view["spec"], view["params"])
    rays = o["tap_rays"]
    pos = o["u2"][rays]                                     # [n, 32, 3], bit-exact vs the oracle
    assert _check_rows(o["rows2"], pos, model.grid, "grid (k_final)") == 1.0
    if view["with_sam"]:
        assert _check_rows(o["srows"], pos, model.s_grid, "s_grid (k_sgrid_box4)") > 0.99
    else:
        assert (o["srows"] == -1).all()


def test_taps_leave_outputs_unchanged(view, cuda):
    """The tapped render (the taps' stores: k_final's and k_sgrid_box4's TAP
    instantiations) gives the product render's outputs bit for bit, and the
    tiled product render (the bench's launch, view_width = W) equals the
    untiled one on the whole 512x512 view."""
    from samnerf_amd.fused import FusedRenderer
    net = make_net(view["spec"], view["params"], cuda)
    fr = FusedRenderer(net)
    ro, rd = view["ro"].to(cuda), view["rd"].to(cuda)
    tiled = fr.render(ro, rd, view_width=W)
    untiled = fr.render(ro, rd)
    for k in ("image", "depth", "weights_sum") + (("samvit",) if view["with_sam"] else ()):
        assert torch.equal(tiled[k].cpu(), view["out"][k]), k
        assert torch.equal(untiled[k].cpu(), view["out"][k]), k
