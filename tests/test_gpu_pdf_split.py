"""k_prop_pdf's split phase A (raymarch.hip prop_pdf_phases, SAMNERF_PDF_SPLIT,
round 6): the two double cumulative sums of the proposal pdf
(nerf/renderer.py:84-119 sample_pdf's cdf, :310-326 compositing's
transmittance) run as quarter prefix sums over the block's four waves when
the ray's terms pass the exact-sum window, and as the sequential chain
otherwise.  Bit for bit the sequential form (the diagnostic build with
SAMNERF_PDF_SEQ=1 forces every ray onto it): composited weights, resampled
bins and searchsorted indices of both proposal stages and the rendered
outputs, on the bench's default-init fog, the parity-weight scene and the
opaque sphere (every ray of all three passes the window: the fast path), and
on a scene whose proposal densities span many decades (the proposal MLPs' output
rows scaled by 1000: most rays fail it, the sequential fallback); the window
fraction per scene is printed (the fast path's share)."""
import numpy as np
import pytest
import torch

from helpers import make_net
from samnerf_amd import synth

pytestmark = pytest.mark.gpu

H = W = 96


def _exact_window(ds):
    """Per ray: do its ds terms (all but the last) pass SumWindow?"""
    a = ds[:, :-1].numpy().astype(np.float32)
    bits = a.view(np.uint32)
    e = (bits >> 23) & 0xFF
    nz = (bits & 0x7FFFFFFF) != 0
    bad = (nz & ((e == 0) | (e == 0xFF))).any(axis=1)
    emax = np.where(nz, e, 0).max(axis=1)
    emin = np.where(nz, e, 0xFF).min(axis=1)
    ok = ~bad & ((emax < emin) | (emax.astype(np.int64) - emin <= 22))
    return ok


@pytest.mark.parametrize("scene", ["default_fog", "parity_weights", "surface", "wide_density"])
def test_split_phase_a_bit_identical_to_sequential(hip_lib, cuda, monkeypatch, scene):
    from samnerf_amd import _lib, ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True)
    if scene == "surface":
        params = synth.make_surface_params(spec, seed=3, amp=1.5)
    else:
        params = synth.make_params(spec, seed=7, emb_scale=1e-4 if scene == "default_fog" else 0.5,
                                   ln_jitter=0.0)
    net = make_net(spec, params, cuda)
    if scene == "wide_density":
        with torch.no_grad():
            for p in range(2):
                net.prop_mlp[p].net[1].weight.mul_(1000.0)
    pose, intr = synth.gui_camera(W, H, rot=synth.random_rotation(6))
    ro, rd = ops.get_rays(pose, intr, H, W, device=cuda)
    prod = FusedRenderer(net).render(ro, rd, taps=True, view_width=W)
    monkeypatch.setenv("SAMNERF_PDF_SEQ", "1")
    with _lib.diag_library():
        seq = FusedRenderer(net).render(ro, rd, taps=True, view_width=W)
    monkeypatch.delenv("SAMNERF_PDF_SEQ")
    torch.cuda.synchronize()
    for k in ("w0", "w1", "bins1", "bins2", "inds1", "inds2", "image", "depth", "weights_sum", "samvit"):
        assert torch.equal(prod[k], seq[k]), (scene, k)
    ok0 = _exact_window(prod["ds0"].cpu())
    ok1 = _exact_window(prod["ds1"].cpu())
    print(f"{scene}: rays on the split path, stage 0 {ok0.mean():.4f}, stage 1 {ok1.mean():.4f}")
    if scene == "default_fog":
        assert ok0.mean() > 0.99 and ok1.mean() > 0.99
    if scene == "wide_density":
        assert min(ok0.mean(), ok1.mean()) < 0.9         # the sequential fallback runs


def test_split_phase_a_nan_density(hip_lib, cuda, monkeypatch):
    """A NaN density (every sigma of one MLP output row): no ray passes the
    window, every ray takes the sequential chain, same bits as forcing it."""
    from samnerf_amd import _lib, ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=False)
    net = make_net(spec, synth.make_params(spec, seed=5, emb_scale=0.5), cuda)
    with torch.no_grad():
        net.prop_mlp[0].net[1].weight[0, :4].fill_(float("nan"))
    pose, intr = synth.gui_camera(32, 32, rot=synth.random_rotation(1))
    ro, rd = ops.get_rays(pose, intr, 32, 32, device=cuda)
    prod = FusedRenderer(net).render(ro, rd, taps=True, view_width=32)
    monkeypatch.setenv("SAMNERF_PDF_SEQ", "1")
    with _lib.diag_library():
        seq = FusedRenderer(net).render(ro, rd, taps=True, view_width=32)
    for k in ("w0", "bins1", "inds1", "w1", "bins2", "inds2"):
        a, b = prod[k], seq[k]
        same = torch.equal(a, b) if not a.is_floating_point() else \
            bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all())
        assert same, k


def test_sgrid_box4_path_counters_cover_every_level_sample(hip_lib, cuda, monkeypatch):
    """The diagnostic build's k_sgrid_box4 path counters (SAMNERF_SGRID_PATHS,
    tools/sgrid_paths.py): every (wave, sample, level) of a view is counted in
    exactly one of the uniform / box / direct paths, or skipped with its wave's
    sample; the render's outputs equal the product's (the counters only add
    atomics in the diagnostic build)."""
    from samnerf_amd import _lib, ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=7, emb_scale=0.5, ln_jitter=0.0), cuda)
    h = w = 256                                            # N >= 32768: the box form runs
    pose, intr = synth.gui_camera(w, h, rot=synth.random_rotation(6))
    ro, rd = ops.get_rays(pose, intr, h, w, device=cuda)
    prod = FusedRenderer(net).render(ro, rd, view_width=w)
    cnt = torch.zeros(8, dtype=torch.int64, device=cuda)
    monkeypatch.setenv("SAMNERF_SGRID_PATHS", f"{cnt.data_ptr():x}")
    with _lib.diag_library():
        diag = FusedRenderer(net).render(ro, rd, view_width=w)
    monkeypatch.delenv("SAMNERF_SGRID_PATHS")
    torch.cuda.synchronize()
    c = cnt.cpu().tolist()
    groups = (h * w) // 64
    # per 64-ray group: 4 level groups x 32 samples (4 quarter-waves x 8), each
    # counted once per level (4) or once as a skipped wave-sample of its group
    assert c[0] + c[1] + c[2] + 4 * c[3] == groups * 32 * 16, c
    assert c[1] > 0, c
    assert c[4] >= c[5] > 0, c                             # padded slots >= cells of the staged boxes
    for k in ("image", "depth", "weights_sum", "samvit"):
        assert torch.equal(prod[k], diag[k]), k
