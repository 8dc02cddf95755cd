"""Hand-off of rendered SAM features to a SAM mask decoder.

`Trainer.sam_predict` (nerf/utils.py:1409-1475) feeds the 256-d feature map
rendered by the NeRF (here: the fused HIP path's `samvit`, already in device
memory) to segment-anything's `SamPredictor` in place of the ViT image
embedding: resize to a 64-long side, zero-pad to 64 x 64, set the
predictor's image state, scale the click to the 1024-long input frame, and
decode one mask.  The decoder itself is a third-party model absent from this
image (segment_anything_hq, requirements.txt:25); `sam_predict` drives any
object with SamPredictor's interface (reset_image, original_size, input_size,
features, is_image_set, interm_features, predict_torch), so a ROCm build of
SAM plugs in unchanged.  Nothing leaves the device: the features stay the
render's tensor, resized and padded on the GPU.
"""
import numpy as np
import torch
import torch.nn.functional as F


def input_size_for(H, W):
    """The predictor's input frame (utils.py:1415-1416): longest side 1024."""
    r = 1024 / W if W > H else 1024 / H
    return (int(H * r), int(W * r)), r


def prepare_sam_features(features):
    """features [1,256,h,w] (or a rendered samvit [h,w,256]) -> [1,256,64,64]:
    bilinear resize of the longest side to 64 (align_corners=False), then
    zero padding right / bottom (utils.py:1426-1431)."""
    if features.dim() == 3:
        features = features.permute(2, 0, 1).unsqueeze(0)
    h, w = features.shape[2:]
    r = 64 / w if w > h else 64 / h
    features = F.interpolate(features, (int(h * r), int(w * r)), mode="bilinear",
                             align_corners=False)
    return F.pad(features, (0, 64 - features.shape[3], 0, 64 - features.shape[2]),
                 mode="constant", value=0)


def click_coords(H, W, point_coords=None, rng=None):
    """Point prompt in the 1024 frame (utils.py:1435-1446): the given pixel
    clicks scaled by the resize ratio, or one random point away from the 20%
    border (np.random, as the reference, unless `rng` is given)."""
    input_size, r = input_size_for(H, W)
    if point_coords is None:
        rng = np.random if rng is None else rng
        bh, bw = int(input_size[0] * 0.2), int(input_size[1] * 0.2)
        # the reference draws x from the height range and y from the width range
        return np.array([[rng.randint(0 + bh, input_size[1] - bh),
                          rng.randint(0 + bw, input_size[0] - bw)]]), r
    return (np.asarray(point_coords).astype(np.float32) * r).astype(np.int32), r


def sam_predict(predictor, H, W, features, point_coords=None, mask_input=None, device=None,
                rng=None):
    """Trainer.sam_predict with rendered features (image=None branch).
    Returns (masks[0] [H, W], original_point_coords [N, 2], low_res_masks[0])."""
    device = device if device is not None else features.device
    input_size, r = input_size_for(H, W)
    predictor.reset_image()
    predictor.original_size = (H, W)
    predictor.input_size = input_size
    predictor.features = prepare_sam_features(features)
    predictor.is_image_set = True
    pts, _ = click_coords(H, W, point_coords, rng)
    mask_t = None
    if mask_input is not None:
        mask_t = torch.as_tensor(mask_input, dtype=torch.float, device=device)[None, :, :, :]
    labels = np.ones_like(pts[:, 0])
    coords_t = torch.as_tensor(pts, dtype=torch.float, device=device)[None, :, :]
    labels_t = torch.as_tensor(labels, dtype=torch.int, device=device)[None, :]
    predictor.interm_features = None
    masks, _iou, low_res = predictor.predict_torch(coords_t, labels_t, mask_input=mask_t,
                                                   multimask_output=False)
    original = (pts / r).astype(np.int32)
    return masks[0], original, low_res[0]


def render_and_predict(renderer, predictor, rays_o_lr, rays_d_lr, h, w, H, W, point_coords=None,
                       **kw):
    """The interactive loop of the GUI (nerf/gui.py:143-161, utils.py:1647-1712)
    on the fused path: render the h x w feature rays, hand the feature map to
    the decoder without a host copy."""
    out = renderer.render(rays_o_lr, rays_d_lr)
    feats = out["samvit"].view(h, w, 256)
    return sam_predict(predictor, H, W, feats, point_coords=point_coords, **kw), out
