#!/usr/bin/env python3
"""Generate tests/golden/sam_bridge.npz from the REFERENCE's Trainer.sam_predict.

Calls nerf/utils.py:1409-1475 (Trainer.sam_predict, unbound) on a minimal
`self` whose `sam_predictor` is a recorder with SamPredictor's interface (the
real SAM decoder, segment_anything_hq, is not installed), and stores what the
reference hands to the decoder: the resized / padded feature map, the
predictor's original / input sizes, the point prompt and labels, and the
returned original-frame click.  Runs only in the build container.

usage: PYTHONDONTWRITEBYTECODE=1 python tools/make_golden_sam_bridge.py
"""
import os
import sys
import types

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402


class Recorder:
    """SamPredictor's interface (reset_image / predict_torch), recording."""

    def reset_image(self):
        self.reset = True

    def predict_torch(self, coords, labels, mask_input=None, multimask_output=True):
        self.coords, self.labels, self.mask_input = coords, labels, mask_input
        self.multimask = multimask_output
        H, W = self.original_size
        f = self.features
        masks = (f.mean(1, keepdim=True)[..., :1, :1] > 0).expand(1, 1, H, W)
        return masks, torch.ones(1, 1), f[:, :1, :, :]


def main():
    mg.install_reference()
    import importlib
    utils = importlib.import_module("nerf.utils")
    out = {}
    g = torch.Generator().manual_seed(3)
    cases = [(512, 512, 64, 64, [[100, 300]]), (480, 640, 48, 64, [[10, 20], [300, 200]]),
             (640, 360, 64, 36, None)]
    for i, (H, W, h, w, pts) in enumerate(cases):
        feats = torch.randn(1, 16, h, w, generator=g)          # the resize is per channel
        rec = Recorder()
        fake = types.SimpleNamespace(sam_predictor=rec, device="cpu")
        np.random.seed(100 + i)
        pc = None if pts is None else np.array(pts, np.int32)
        masks, orig, low = utils.Trainer.sam_predict(fake, H, W, feats, point_coords=pc)
        out[f"c{i}_in"] = feats.numpy()
        out[f"c{i}_HW"] = np.array([H, W])
        out[f"c{i}_pts"] = np.array(pts if pts is not None else [[-1, -1]], np.int32)
        out[f"c{i}_seed"] = np.array(100 + i)
        out[f"c{i}_features"] = rec.features.numpy()
        out[f"c{i}_sizes"] = np.array([*rec.original_size, *rec.input_size])
        out[f"c{i}_coords"] = rec.coords.numpy()
        out[f"c{i}_labels"] = rec.labels.numpy()
        out[f"c{i}_orig"] = np.asarray(orig)
        out[f"c{i}_multimask"] = np.array(rec.multimask)
        print(f"  case {i}: H,W={H},{W} features {tuple(rec.features.shape)} coords "
              f"{rec.coords.numpy().tolist()} input_size {rec.input_size}")
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "sam_bridge.npz"), **out)


if __name__ == "__main__":
    main()
