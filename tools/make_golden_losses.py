#!/usr/bin/env python3
"""Generate tests/golden/losses.npz from the REFERENCE's proposal_loss.

`proposal_loss` (nerf/renderer.py:30-57) is pure torch and is imported from the
reference (with the stubs of make_golden.py).  `distort_loss` calls the
third-party `torch_efficient_distloss.eff_distloss`, which is absent from the
container (un-pinned in requirements.txt:22); the stub cannot compute it, so
its parity is unpinned and tests/test_losses.py pins the restatement against
the loss's defining double sum instead.

usage: PYTHONDONTWRITEBYTECODE=1 python tools/make_golden_losses.py
"""
import os
import sys

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402


def sorted_bins(g, n, t):
    b = torch.sort(torch.rand(n, t + 1, generator=g, dtype=torch.float32), dim=-1).values
    b[:, 0] = 0.0
    b[:, -1] = 1.0
    return b


def main():
    _, renderer, _ = mg.install_reference()
    g = torch.Generator().manual_seed(7)
    n = 64
    out = {}
    bins = [sorted_bins(g, n, 128), sorted_bins(g, n, 64), sorted_bins(g, n, 32)]
    weights = [torch.rand(n, t, generator=g) / t for t in (128, 64, 32)]
    weights[0][3] = 0.0                                  # an all-zero row
    loss = renderer.proposal_loss(bins, weights)
    for i in range(3):
        out[f"bins{i}"] = bins[i].numpy()
        out[f"weights{i}"] = weights[i].numpy()
    out["proposal_loss"] = np.array(float(loss), dtype=np.float32)
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "losses.npz"), **out)
    print("losses.npz written: proposal_loss =", float(loss))


if __name__ == "__main__":
    main()
