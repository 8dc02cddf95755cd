"""Training losses of the RGB stage and the CPU twin of the
unfused training path.  CPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from helpers import make_net
from oracle import synth


def test_proposal_loss_matches_reference_golden():
    """tests/golden/losses.npz holds the reference's own proposal_loss
    (renderer.py:30-57, tools/make_golden_losses.py) on random inputs incl.
    an all-zero weight row."""
    from nerf.renderer import proposal_loss
    g = np.load(os.path.join(GOLDEN, "losses.npz"))
    bins = [torch.from_numpy(g[f"bins{i}"]) for i in range(3)]
    weights = [torch.from_numpy(g[f"weights{i}"]) for i in range(3)]
    loss = proposal_loss(bins, weights)
    assert float(loss) == float(g["proposal_loss"])


def test_distort_loss_equals_its_definition():
    """eff_distloss restates a third-party function absent here (parity
    unpinned): pin its O(T) form to the defining double sum
    sum_ij w_i w_j |m_i - m_j| + 1/3 sum_i w_i^2 s_i, mean over rays."""
    from nerf.renderer import distort_loss
    g = torch.Generator().manual_seed(3)
    b = torch.sort(torch.rand(16, 33, generator=g, dtype=torch.float64), -1).values
    w = torch.rand(16, 32, generator=g, dtype=torch.float64) / 32
    s = b[:, 1:] - b[:, :-1]
    m = b[:, :-1] + s / 2
    brute = ((w[:, :, None] * w[:, None, :] * (m[:, :, None] - m[:, None, :]).abs()).sum((1, 2))
             + (w ** 2 * s).sum(-1) / 3).mean()
    assert torch.allclose(distort_loss(b, w), brute, rtol=1e-12, atol=0)


def test_training_extras_on_cpu_twin():
    """run_torch in training mode returns the reference's extras
    (renderer.py:348-356): proposal / distortion losses, num_points, weights,
    and a backward pass reaches every RGB parameter (CPU twin: oracle
    encoders)."""
    from oracle_backend import oracle_encoders
    from samnerf_amd.train import rgb_train_step
    spec = synth.ModelSpec(with_sam=False, grid_log2=10, s_grid_log2=10, prop_log2=9)
    net = make_net(spec, synth.make_params(spec, seed=2, emb_scale=0.5), "cpu")
    net.fused = False
    net.train()
    pose, intr = synth.gui_camera(8, 8, rot=synth.random_rotation(1))
    from oracle import renderer as orc
    ro, rd = orc.get_rays(pose, intr, 8, 8)
    gt = torch.rand(64, 3, generator=torch.Generator().manual_seed(0))
    with oracle_encoders():
        pred, loss, out = rgb_train_step(net, ro, rd, gt, global_step=1, perturb=False)
        assert {"proposal_loss", "distort_loss", "num_points", "weights"} <= set(out)
        assert out["num_points"] == 64 * 32
        loss.backward()
    grads = {k: p.grad for k, p in net.named_parameters()}
    for k in ("grid.embeddings", "grid_mlp.net.0.weight", "view_mlp.net.2.weight",
              "prop_encoders.0.embeddings", "prop_mlp.1.net.1.weight"):
        assert grads[k] is not None and grads[k].abs().sum() > 0, k
    # adaptive ray count (utils.py:933-935): num_points / points used * num_rays
    assert net.opt.num_rays == int(round(2 ** 18 / (64 * 32) * 4096))
