"""N1, the flagged non-parity early-exit mode (samnerf_model.
t_thresh), on a scene whose rays saturate: synth.make_surface_params' opaque
sphere (random weights never get there -- their transmittance stays above
1e-2 until the last sample, which absorbs the rest).

The same scene is also a parity case of its own for the default mode: sharp
density, proposal resampling concentrated at the surface.
"""
import numpy as np
import pytest
import torch

from helpers import make_net, max_abs, oracle_for
from samnerf_amd import synth

pytestmark = pytest.mark.gpu

H = W = 48


def _scene(cuda):
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_surface_params(spec, seed=3, amp=1.5)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(W, H, rot=synth.random_rotation(6))
    from oracle import renderer as orc
    ro, rd = orc.get_rays(pose, intr, H, W)
    ref = oracle_for(spec, params).run(ro, rd, return_feats=1)
    return net, ro.to(cuda), rd.to(cuda), ref


@pytest.fixture(scope="module")
def scene(cuda):
    return _scene(cuda)


def _render(net, ro, rd, t_thresh):
    from samnerf_amd.fused import FusedRenderer
    out = FusedRenderer(net, t_thresh=t_thresh).render(ro, rd)
    return {k: v.cpu() for k, v in out.items()}


def test_surface_scene_default_mode_matches_oracle(hip_lib, scene):
    net, ro, rd, ref = scene
    out = _render(net, ro, rd, 0.0)
    d_rel = ((out["depth"] - ref["depth"]).abs() / ref["depth"].abs().clamp(min=1.0)).max().item()
    errs = {"image": max_abs(out["image"], ref["image"]), "wsum": max_abs(out["weights_sum"], ref["weights_sum"]),
            "depth_rel": d_rel, "samvit": max_abs(out["samvit"], ref["samvit"])}
    print("surface scene, default mode vs oracle", errs)
    assert max(errs.values()) < 1e-3, errs


@pytest.mark.parametrize("t", [1e-4, 1e-3])
def test_early_exit_error_bounded_by_threshold(hip_lib, scene, t):
    """Dropped samples carry at most t of each ray's weight: weights_sum falls
    by at most t, image moves by at most t x |colour - background| <= t,
    depth by at most t x the ray's far distance; samvit (LayerNorm head) is
    reported and held to 100 t.  Some waves must actually have exited."""
    net, ro, rd, ref = scene
    full = _render(net, ro, rd, 0.0)
    out = _render(net, ro, rd, t)
    exited = (out["weights_sum"] < 1.0 - 1e-6)
    d_err = (out["depth"] - full["depth"]).abs()
    from oracle import renderer as orc
    _, far = orc.near_far_from_aabb(ro.cpu(), rd.cpu(), torch.tensor([-128.0] * 3 + [128.0] * 3), 0.2)
    errs = {"exited_rays": exited.float().mean().item(),
            "wsum_drop": (full["weights_sum"] - out["weights_sum"]).max().item(),
            "image_vs_oracle": max_abs(out["image"], ref["image"]),
            "depth_over_far": (d_err / far).max().item(),
            "samvit_vs_oracle": max_abs(out["samvit"], ref["samvit"])}
    print("N1", t, errs)
    assert errs["exited_rays"] > 0.1, errs
    assert errs["wsum_drop"] <= t * 1.001 + 1e-6
    assert errs["image_vs_oracle"] <= t + 1e-3
    assert errs["depth_over_far"] <= t * 1.001 + 1e-6
    assert errs["samvit_vs_oracle"] <= 100 * t + 1e-3
    # the mode is opt-in: a renderer without it reproduces the default bits
    again = _render(net, ro, rd, 0.0)
    assert all(torch.equal(again[k], full[k]) for k in full)


def _full_one_segment(net, ro, rd, monkeypatch):
    """The default mode at N1's one segment per ray (small views split their
    rays into 2 or 4 segments by default: another summation order)."""
    from samnerf_amd import _lib
    monkeypatch.setenv("SAMNERF_FINAL_S", "1")
    with _lib.diag_library():
        out = _render(net, ro, rd, 0.0)
    monkeypatch.delenv("SAMNERF_FINAL_S")
    return out


def test_compaction_exact_when_no_ray_closes(hip_lib, cuda, monkeypatch, diag):
    """N1's ray compaction (k_final passes over 8-sample chunks; the rays still
    open at a chunk's end -- wave ballot, scan, scatter -- form the next
    pass's list, their running sums carried in the workspace): on a
    parity-weight scene no ray's transmittance falls below 1e-4 before its
    last sample, so every ray goes through all four passes and the render
    must equal the default mode's bits.  (The passes are the diagnostic
    build's SAMNERF_N1_CHUNKS; the product's N1 is the wave-level exit,
    measured faster, profiles/r3_n1_compaction.txt.)"""
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    net = make_net(spec, synth.make_params(spec, seed=4, emb_scale=0.5), cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(2))
    from oracle import renderer as orc
    ro, rd = orc.get_rays(pose, intr, 64, 64)
    ro, rd = ro.to(cuda), rd.to(cuda)
    from samnerf_amd import _lib
    full = _full_one_segment(net, ro, rd, monkeypatch)
    monkeypatch.setenv("SAMNERF_N1_CHUNKS", "4")
    with _lib.diag_library():
        out = _render(net, ro, rd, 1e-4)
    for k in ("image", "depth", "weights_sum", "samvit"):
        assert torch.equal(out[k], full[k]), k


@pytest.mark.parametrize("chunks", ["2", "4", "8"])
def test_compaction_error_bounded_by_threshold(hip_lib, scene, monkeypatch, diag, chunks):
    """The diagnostic build's compaction passes (2 / 4 / 8 sample chunks) on
    the opaque-sphere scene: the same bound as the wave-level exit -- each
    ray loses at most t of its weight -- and rays do close."""
    from samnerf_amd import _lib
    net, ro, rd, ref = scene
    t = 1e-3
    full = _full_one_segment(net, ro, rd, monkeypatch)
    monkeypatch.setenv("SAMNERF_N1_CHUNKS", chunks)
    with _lib.diag_library():
        out = _render(net, ro, rd, t)
    drop = full["weights_sum"] - out["weights_sum"]
    assert (drop > 0).float().mean().item() > 0.1
    assert drop.max().item() <= t * 1.001 + 1e-6
    assert max_abs(out["image"], ref["image"]) <= t + 1e-3


def _align256(nbytes):
    return (nbytes + 255) // 256 * 256


def test_early_exit_nan_sigma_stays_in_its_segment(hip_lib, cuda):
    """a small view's rays are cut into 4 segments of 8
    steps (N < 32768), and k_final's N1 form must stop at 8 steps even when no
    ray ever closes -- here every sigma is NaN (cum NaN never exceeds
    -ln t).  The head-input rows region, which follows the final weights in
    the workspace (raymarch.hip carve) and is unused by an RGB-only render,
    is filled with a canary that must survive."""
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=False, grid_log2=14, prop_log2=12)
    net = make_net(spec, synth.make_params(spec, seed=5, emb_scale=0.5), cuda)
    from oracle import renderer as orc
    pose, intr = synth.gui_camera(W, H, rot=synth.random_rotation(1))
    ro, rd = orc.get_rays(pose, intr, H, W)
    ro, rd = ro.to(cuda), rd.to(cuda)
    N = ro.shape[0]
    assert N < 32768                                     # 4 segments per ray
    fr = FusedRenderer(net, t_thresh=1e-3)
    ws = fr.render(ro, rd, keep_workspace=True)["_workspace"][0]
    with torch.no_grad():
        net.grid_mlp.net[2].weight[0].fill_(float("nan"))   # sigma row of grid_mlp's last layer
    # carve(): the N-independent packed weights first (gpack 2 x 16 slots x 64
    # lanes x 4 words, gexp 4 floats, no SAM head), then snf 2N, rec 8N,
    # bins1 65N, bins2 33N, wtmp 128N, u_f 96N, w_f 32N, rows 164N floats
    off = _align256(4 * 2 * 16 * 64 * 4) + _align256(4 * 4)
    off += sum(_align256(4 * f * N) for f in (2, 8, 65, 33, 128, 96, 32))
    region = ws[off:off + 4 * 164 * N]
    region.fill_(0x5A)
    out = fr.render(ro, rd, keep_workspace=True)
    torch.cuda.synchronize()
    assert out["_workspace"][0].data_ptr() == ws.data_ptr()
    assert bool((region == 0x5A).all()), "k_final wrote past its segment's steps"
    print("NaN-sigma N1 render: weights_sum range", out["weights_sum"].min().item(), out["weights_sum"].max().item())
