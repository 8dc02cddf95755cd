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
  flip where u_j lies within an ulp of a cdf entry.
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
    out = FusedRenderer(net).render(ro, rd, taps=True)
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
