"""Host-side widening of the path: reference checkpoints and
the COLMAP camera convention.  CPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from helpers import make_net
from oracle import synth


# ------------------------------------------------------------- cameras --

@pytest.mark.parametrize("case", [0, 1, 2])
def test_colmap_to_nerf_matches_reference(case):
    """tests/golden/cameras.npz was made by the reference's own qvec2rotmat /
    rotmat / center_poses (tools/make_golden_cameras.py); the restatement is
    bit-identical (same float64 op order)."""
    from samnerf_amd import scene
    g = np.load(os.path.join(GOLDEN, "cameras.npz"))
    p = f"c{case}_"
    poses, pts, s = scene.colmap_to_nerf(g[p + "q"], g[p + "t"], g[p + "pts"],
                                         scale=float(g[p + "scale_in"]),
                                         enable_cam_center=bool(g[p + "cam_center"]))
    np.testing.assert_array_equal(poses, g[p + "poses"])
    np.testing.assert_array_equal(pts, g[p + "pts_out"])
    assert s == float(g[p + "scale"])
    np.testing.assert_array_equal(scene.qvec2rotmat(g[p + "q"][0]), g[p + "rot0"])
    np.testing.assert_array_equal(scene.rotmat(np.array([0.3, -0.2, 0.9]), [0, 0, 1]), g[p + "rotmat"])
    # camera-to-world rotations stay orthonormal; cameras end up inside the unit ball
    R = poses[:, :3, :3]
    np.testing.assert_allclose(R @ R.transpose(0, 2, 1), np.broadcast_to(np.eye(3), R.shape), atol=1e-9)  # rotmat adds 1e-10 to a denominator
    if float(g[p + "scale_in"]) == -1:
        assert np.linalg.norm(poses[:, :3, 3], axis=-1).max() == pytest.approx(1.0)


def test_colmap_intrinsics_and_sam_grid():
    from samnerf_amd import scene
    np.testing.assert_array_equal(scene.colmap_intrinsics("PINHOLE", [800.0, 810.0, 320.0, 240.0], 2),
                                  np.array([400, 405, 160, 120], np.float32))
    np.testing.assert_array_equal(scene.colmap_intrinsics("SIMPLE_RADIAL", [700.0, 300.0, 200.0, 0.1]),
                                  np.array([700, 700, 300, 200], np.float32))
    with pytest.raises(ValueError):
        scene.colmap_intrinsics("FOV", [1.0] * 5)
    f = 512 / (2 * np.tan(0.5 * 60 * np.pi / 180))
    np.testing.assert_array_equal(scene.sam_view_intrinsics(512), np.array([f, f, 256, 256], np.float32))
    assert scene.sam_feature_grid(512) == (8, 64)       # the 64x64 feature rays of cfg 5
    assert scene.sam_feature_grid(1024) == (16, 64)


# ---------------------------------------------------------- checkpoints --

def _net(seed):
    spec = synth.ModelSpec(with_sam=True, grid_log2=10, s_grid_log2=10, prop_log2=9)
    return make_net(spec, synth.make_params(spec, seed=seed, emb_scale=0.5), "cpu")


def _same(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    return sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sa)


def test_checkpoint_roundtrip_reference_layout(tmp_path):
    """Model-only checkpoint in the reference's layout (utils.py:2046-2074),
    read back with weights_only=True, restores every tensor incl. offsets."""
    from samnerf_amd import checkpoint as ck
    src, dst = _net(1), _net(2)
    assert not _same(src, dst)
    path = tmp_path / "ngp_ep0007.pth"
    ck.save_checkpoint(src, path, epoch=7, global_step=1234)
    raw = ck.read_checkpoint(path)
    assert set(raw) == {"epoch", "global_step", "stats", "model"}
    assert "grid.offsets" in raw["model"] and raw["model"]["grid.offsets"].dtype == torch.int32
    info = ck.load_checkpoint(dst, str(path))
    assert info["missing"] == [] and info["unexpected"] == []
    assert info["epoch"] == 7 and info["global_step"] == 1234
    assert _same(src, dst)
    assert ck.latest_checkpoint(tmp_path) == str(path)
    assert ck.latest_checkpoint(tmp_path / "none") is None


def test_checkpoint_bare_state_dict_and_partial(tmp_path):
    from samnerf_amd import checkpoint as ck
    src, dst = _net(3), _net(4)
    torch.save(src.state_dict(), tmp_path / "bare.pth")
    ck.load_checkpoint(dst, str(tmp_path / "bare.pth"))            # strict, as the reference
    assert _same(src, dst)
    sd = {k: v for k, v in src.state_dict().items() if not k.startswith("samvit_mlp")}
    sd["extra.weight"] = torch.zeros(1)
    info = ck.load_checkpoint(_net(5), {"model": sd, "epoch": 1, "global_step": 2})
    assert any(k.startswith("samvit_mlp") for k in info["missing"])
    assert info["unexpected"] == ["extra.weight"]
    with pytest.raises(RuntimeError):                                  # strict bare dict
        ck.load_checkpoint(_net(6), sd)


def test_checkpoint_ema_copy_to(tmp_path):
    """use_ema renders with the EMA shadow weights (utils.py:1684-1686), for
    shadows over all parameters or over the trainable subset only."""
    from samnerf_amd import checkpoint as ck
    src = _net(7)
    shadow = [p.detach() + 0.25 for p in src.parameters()]
    ck.save_checkpoint(src, tmp_path / "e.pth", ema_shadow=shadow)
    dst = _net(8)
    ck.load_checkpoint(dst, str(tmp_path / "e.pth"), use_ema=True)
    for p, s in zip(dst.parameters(), shadow):
        assert torch.equal(p, s)
    # older torch_ema: shadow over requires_grad parameters only (RGB frozen)
    dst2 = _net(9)
    for n, p in dst2.named_parameters():
        p.requires_grad_(n.startswith("s_grid") or n.startswith("samvit_mlp"))
    trainable = [p for p in dst2.parameters() if p.requires_grad]
    sub = [p.detach() - 1.0 for p in trainable]
    ck.load_checkpoint(dst2, {"model": src.state_dict(), "ema": {"shadow_params": sub}}, use_ema=True)
    for p, s in zip(trainable, sub):
        assert torch.equal(p, s)
    with pytest.raises(ValueError):
        ck.load_checkpoint(_net(10), {"model": src.state_dict(), "ema": {"shadow_params": sub[:2]}},
                           use_ema=True)
