#!/usr/bin/env python3
"""Generate tests/golden/cameras.npz from the REFERENCE's camera code.

Imports nerf/colmap_provider.py (for `rotmat`, `center_poses`) and
nerf/colmap_utils.py (`qvec2rotmat`) from /root/reference with inert stubs for
the third-party modules it imports but these functions do not use (cv2,
trimesh, pyquaternion, ...); the reference's CUDA encoders are never imported.
The pose pipeline of ColmapDataset.__init__ (colmap_provider.py:490-528) is
inline code in the reference, so it is transcribed here step by step around
the reference's own functions.  Runs only in the build container.

usage: PYTHONDONTWRITEBYTECODE=1 python tools/make_golden_cameras.py
"""
import os
import sys

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402  (stub helpers, install_reference)


def main():
    for n in ["pyquaternion"]:
        mg._stub(n)
    mg.install_reference()
    import importlib
    cp = importlib.import_module("nerf.colmap_provider")
    cu = importlib.import_module("nerf.colmap_utils")
    rng = np.random.default_rng(11)
    out = {}
    for case, (n_cam, n_pts, cam_center, scale) in enumerate(
            [(6, 40, False, -1.0), (9, 25, True, -1.0), (5, 30, False, 0.37)]):
        q = rng.normal(size=(n_cam, 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        t = rng.normal(size=(n_cam, 3)) * 3.0
        pts = rng.normal(size=(n_pts, 3)) * 2.0 + 0.5
        # colmap_provider.py:490-501
        poses = []
        for k in range(n_cam):
            P = np.eye(4, dtype=np.float64)
            P[:3, :3] = cu.qvec2rotmat(q[k])
            P[:3, 3] = t[k]
            poses.append(P)
        poses = np.linalg.inv(np.stack(poses, axis=0))
        # :512
        poses_c, pts_c = cp.center_poses(poses.copy(), pts.copy(), cam_center)
        # :515-520
        poses_c[:, :3, 1:3] *= -1
        poses_c = poses_c[:, [1, 0, 2, 3], :]
        poses_c[:, 2] *= -1
        pts_c = pts_c[:, [1, 0, 2]]
        pts_c[:, 2] *= -1
        # :522-528
        s = scale
        if s == -1:
            s = 1 / np.linalg.norm(poses_c[:, :3, 3], axis=-1).max()
        poses_c[:, :3, 3] *= s
        pts_c = pts_c * s
        out[f"c{case}_q"], out[f"c{case}_t"], out[f"c{case}_pts"] = q, t, pts
        out[f"c{case}_cam_center"] = np.array(cam_center)
        out[f"c{case}_scale_in"] = np.array(scale)
        out[f"c{case}_poses"], out[f"c{case}_pts_out"], out[f"c{case}_scale"] = poses_c, pts_c, np.array(s)
        out[f"c{case}_rot0"] = cu.qvec2rotmat(q[0])
        out[f"c{case}_rotmat"] = cp.rotmat(np.array([0.3, -0.2, 0.9]), [0, 0, 1])
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "cameras.npz"), **out)
    print("cameras.npz written:", sorted(out)[:6], "...")


if __name__ == "__main__":
    main()
