"""SAM decoder hand-off: samnerf_amd.sam_bridge.sam_predict
hands the decoder exactly what the reference's Trainer.sam_predict
(nerf/utils.py:1409-1475) hands it -- resized / padded features, image sizes,
prompt coordinates and labels -- pinned by tests/golden/sam_bridge.npz, made
by tools/make_golden_sam_bridge.py from the reference's own method."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN


class Recorder:
    def reset_image(self):
        self.reset = True

    def predict_torch(self, coords, labels, mask_input=None, multimask_output=True):
        self.coords, self.labels, self.multimask = coords, labels, multimask_output
        H, W = self.original_size
        f = self.features
        return (f.mean(1, keepdim=True)[..., :1, :1] > 0).expand(1, 1, H, W), torch.ones(1, 1), f[:, :1]


@pytest.mark.parametrize("case", [0, 1, 2])
def test_sam_predict_hands_off_like_the_reference(case):
    from samnerf_amd.sam_bridge import sam_predict
    g = np.load(os.path.join(GOLDEN, "sam_bridge.npz"))
    H, W = [int(v) for v in g[f"c{case}_HW"]]
    pts = g[f"c{case}_pts"]
    pts = None if pts[0, 0] < 0 else pts
    rec = Recorder()
    np.random.seed(int(g[f"c{case}_seed"]))
    masks, orig, low = sam_predict(rec, H, W, torch.from_numpy(g[f"c{case}_in"]), point_coords=pts)
    assert rec.reset and rec.is_image_set and rec.interm_features is None
    assert np.array_equal(rec.features.numpy(), g[f"c{case}_features"])
    assert [*rec.original_size, *rec.input_size] == g[f"c{case}_sizes"].tolist()
    assert np.array_equal(rec.coords.numpy(), g[f"c{case}_coords"])
    assert np.array_equal(rec.labels.numpy(), g[f"c{case}_labels"])
    assert np.array_equal(orig, g[f"c{case}_orig"]) and not rec.multimask
    assert masks.shape == (1, H, W)          # (fixture: 16 channels; the resize is per channel)


def test_rendered_feature_map_layout():
    """A rendered samvit [h, w, 256] is the reference's [1, 256, h, w] map."""
    from samnerf_amd.sam_bridge import prepare_sam_features
    f = torch.randn(1, 256, 48, 64)
    a = prepare_sam_features(f)
    b = prepare_sam_features(f[0].permute(1, 2, 0).contiguous())
    assert torch.equal(a, b) and a.shape == (1, 256, 64, 64)
    assert (a[:, :, 48:] == 0).all()
