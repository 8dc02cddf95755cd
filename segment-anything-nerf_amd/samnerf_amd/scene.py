"""Camera conventions of the reference's COLMAP scenes (host side, numpy).

The fused renderer takes camera-to-world poses and pinhole intrinsics in the
convention `get_rays` (nerf/utils.py:145-279) expects.  For real scenes the
reference's ColmapDataset (nerf/colmap_provider.py) produces them from a
COLMAP reconstruction:

  * intrinsics per camera model (colmap_provider.py:472-487);
  * world-to-camera (qvec, tvec) -> camera-to-world (:490-501);
  * re-centring on the sparse points and rotating the mean camera up-vector to
    +z (`center_poses`, :50-74, with `rotmat` :38-47);
  * the axis convention flip (:513-520) and auto-scale into the box (:522-528);
  * for SAM-feature rendering, square 512-px-style views with a fixed 60-degree
    fovy and the 64x64 feature-ray grid (:989-1004, 1187-1196).

These functions restate those steps (same float64 op order) so a user with a
reconstruction can render its cameras with this package; tests/golden
cameras.npz pins them against the reference's own functions.  Reading the
COLMAP binary files and the images themselves is data-provider work outside
the hot path.
"""
import numpy as np


def qvec2rotmat(qvec):
    """colmap_utils.py:272-282 (w, x, y, z quaternion -> rotation matrix)."""
    return np.array([
        [1 - 2 * qvec[2] ** 2 - 2 * qvec[3] ** 2,
         2 * qvec[1] * qvec[2] - 2 * qvec[0] * qvec[3],
         2 * qvec[3] * qvec[1] + 2 * qvec[0] * qvec[2]],
        [2 * qvec[1] * qvec[2] + 2 * qvec[0] * qvec[3],
         1 - 2 * qvec[1] ** 2 - 2 * qvec[3] ** 2,
         2 * qvec[2] * qvec[3] - 2 * qvec[0] * qvec[1]],
        [2 * qvec[3] * qvec[1] - 2 * qvec[0] * qvec[2],
         2 * qvec[2] * qvec[3] + 2 * qvec[0] * qvec[1],
         1 - 2 * qvec[1] ** 2 - 2 * qvec[2] ** 2]])


def rotmat(a, b, rng=np.random):
    """Rotation taking direction a to direction b (colmap_provider.py:38-47,
    Rodrigues form; the antiparallel case perturbs a randomly, as there)."""
    a, b = a / np.linalg.norm(a), b / np.linalg.norm(b)
    v = np.cross(a, b)
    c = np.dot(a, b)
    if c < -1 + 1e-10:
        return rotmat(a + rng.uniform(-1e-2, 1e-2, 3), b, rng)
    s = np.linalg.norm(v)
    kmat = np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])
    return np.eye(3) + kmat + kmat.dot(kmat) * ((1 - c) / (s ** 2 + 1e-10))


def center_poses(poses, pts3d=None, enable_cam_center=False):
    """colmap_provider.py:50-74.  Modifies `poses` translation in place (as the
    reference does) and returns the centred poses (and points)."""
    def normalize(v):
        return v / (np.linalg.norm(v) + 1e-10)

    if pts3d is None or enable_cam_center:
        center = poses[:, :3, 3].mean(0)
    else:
        center = pts3d.mean(0)
    up = normalize(poses[:, :3, 1].mean(0))
    R = rotmat(up, [0, 0, 1])
    R = np.pad(R, [0, 1])
    R[-1, -1] = 1
    poses[:, :3, 3] -= center
    poses_centered = R @ poses
    if pts3d is not None:
        return poses_centered, (pts3d - center) @ R[:3, :3].T
    return poses_centered


def colmap_intrinsics(model, params, downscale=1):
    """(fx, fy, cx, cy) float32 for a COLMAP camera (colmap_provider.py:474-487)."""
    if model in ("SIMPLE_RADIAL", "SIMPLE_PINHOLE"):
        fl_x = fl_y = params[0] / downscale
        cx, cy = params[1] / downscale, params[2] / downscale
    elif model in ("PINHOLE", "OPENCV"):
        fl_x, fl_y = params[0] / downscale, params[1] / downscale
        cx, cy = params[2] / downscale, params[3] / downscale
    else:
        raise ValueError(f"Unsupported colmap camera model: {model}")
    return np.array([fl_x, fl_y, cx, cy], dtype=np.float32)


def colmap_to_nerf(qvecs, tvecs, pts3d, scale=-1.0, enable_cam_center=False):
    """COLMAP world-to-camera (qvec [N,4], tvec [N,3]) + sparse points [M,3] ->
    (poses [N,4,4] float64 camera-to-world in the renderer's convention,
    pts3d [M,3], scale), as ColmapDataset.__init__ does (colmap_provider.py:
    490-528).  `scale` = -1 picks the auto-scale 1 / max camera distance."""
    poses = []
    for q, t in zip(qvecs, tvecs):
        P = np.eye(4, dtype=np.float64)
        P[:3, :3] = qvec2rotmat(q)
        P[:3, 3] = t
        poses.append(P)
    poses = np.linalg.inv(np.stack(poses, axis=0))
    poses, pts3d = center_poses(poses, np.asarray(pts3d, dtype=np.float64), enable_cam_center)
    poses[:, :3, 1:3] *= -1                       # rectify convention
    poses = poses[:, [1, 0, 2, 3], :]
    poses[:, 2] *= -1
    pts3d = pts3d[:, [1, 0, 2]]
    pts3d[:, 2] *= -1
    if scale == -1:
        scale = 1 / np.linalg.norm(poses[:, :3, 3], axis=-1).max()
    poses[:, :3, 3] *= scale
    pts3d = pts3d * scale
    return poses, pts3d, scale


def sam_view_intrinsics(resolution, fovy=60.0):
    """Square view at the SAM online resolution with a fixed fovy (eval branch
    of colmap_provider.py:989-1004): (fx, fy, cx, cy) float32."""
    focal = resolution / (2 * np.tan(0.5 * fovy * np.pi / 180))
    return np.array([focal, focal, resolution / 2, resolution / 2], dtype=np.float32)


def sam_feature_grid(resolution):
    """Intrinsics divisor and size of the low-resolution feature-ray grid the
    SAM branch renders (colmap_provider.py:1187-1196): 16 * res // 1024 and
    res // that (64 for 512)."""
    scale = 16 * resolution // 1024
    return scale, resolution // scale
