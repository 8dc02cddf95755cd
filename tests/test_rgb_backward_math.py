"""The closed forms the RGB training kernels use for their backward
(csrc/rgb_train.hip), restated in float64 numpy and checked against torch
autograd of the reference's own expressions (nerf/renderer.py:17-57, 309-326
as restated in segment-anything-nerf_amd/nerf/renderer.py) on the CPU:

  * compositing (k_rt_final_bwd_ray_h, k_rt_prop_ray_w): w_k = (1 - e^-ds_k) T_k,
    T_k = exp(-sum_{j<k} ds_j), last ds = +inf (no gradient), nan_to_num_:
    d ds_j = dw_j e^-ds_j T_j - sum_{k>j} dw_k w_k   (reverse scan);
  * distortion (eff_distloss): d/dw_k = 2 (m_k W_<k - WM_<k + WM_>k - m_k W_>k)
    + 2/3 s_k w_k  (per ray; the mean over rays scales it);
  * proposal loss: w = cw1[hi + 1] - cw1[lo] is a signed range sum of the
    stage weights, so its gradient is a difference array (+g at lo, -g at
    hi + 1), whatever the order of lo and hi.
"""
import numpy as np
import torch

from nerf.renderer import distort_loss, proposal_loss


def _composite(ds):
    ds = torch.cat([ds[..., :-1], torch.full_like(ds[..., -1:], torch.inf)], dim=-1)
    alphas = 1 - torch.exp(-ds)
    trans = torch.cumsum(ds[..., :-1], dim=-1)
    trans = torch.exp(-torch.cat([torch.zeros_like(trans[..., :1]), trans], dim=-1))
    w = alphas * trans
    return w.nan_to_num(0)


def _composite_bwd(ds, dw):
    """The kernels' reverse scan, float64 numpy, one ray per row."""
    N, T = ds.shape
    out = np.zeros_like(ds)
    for r in range(N):
        cum = 0.0
        raw = np.zeros(T)
        ev = np.zeros(T)
        for k in range(T):
            d = np.inf if k == T - 1 else ds[r, k]
            e, Tk = np.exp(-d), np.exp(-cum)
            cum += d
            raw[k] = (1 - e) * Tk
            ev[k] = e * Tk
        acc = 0.0
        for k in range(T - 1, -1, -1):
            if k < T - 1:
                out[r, k] = dw[r, k] * ev[k] - acc
            acc += dw[r, k] * raw[k]
    return out


def test_compositing_reverse_scan_matches_autograd():
    g = torch.Generator().manual_seed(0)
    ds = (torch.rand(16, 32, generator=g, dtype=torch.float64) * 0.4).requires_grad_(True)
    dw = torch.randn(16, 32, generator=g, dtype=torch.float64)
    (_composite(ds) * dw).sum().backward()
    ours = _composite_bwd(ds.detach().numpy(), dw.numpy())
    np.testing.assert_allclose(ours, ds.grad.numpy(), rtol=1e-10, atol=1e-12)
    assert (ds.grad[:, -1] == 0).all()                      # the +inf sample has no gradient


def test_distortion_gradient_closed_form():
    g = torch.Generator().manual_seed(1)
    bins = torch.sort(torch.rand(8, 33, generator=g, dtype=torch.float64), dim=-1).values
    w = torch.rand(8, 32, generator=g, dtype=torch.float64).requires_grad_(True)
    distort_loss(bins, w).backward()
    b, wn = bins.numpy(), w.detach().numpy()
    s = b[:, 1:] - b[:, :-1]
    m = b[:, :-1] + s / 2
    W, WM = np.cumsum(wn, 1), np.cumsum(wn * m, 1)
    Wt, WMt = W[:, -1:], WM[:, -1:]
    before = m * (W - wn) - (WM - wn * m)
    after = (WMt - WM) - m * (Wt - W)
    ours = (2 * (before + after) + (2 / 3) * s * wn) / wn.shape[0]
    np.testing.assert_allclose(ours, w.grad.numpy(), rtol=1e-10, atol=1e-13)


def _upper_bound(arr, v):
    lo, hi = 0, len(arr)
    while lo < hi:
        mid = lo + ((hi - lo) >> 1)
        if not (v < arr[mid]):
            lo = mid + 1
        else:
            hi = mid
    return lo


def test_proposal_loss_gradient_is_a_difference_array():
    """One proposal stage against the final one (renderer.py:35-49): the
    kernels' searchsorted (ATen's bisection), the range sums and the
    difference-array gradient, against autograd of proposal_loss."""
    g = torch.Generator().manual_seed(2)
    N, T0, T1 = 6, 32, 64
    t_ref = torch.sort(torch.rand(N, T0 + 1, generator=g, dtype=torch.float64), -1).values
    w_ref = torch.rand(N, T0, generator=g, dtype=torch.float64) * 0.2
    t1 = torch.sort(torch.rand(N, T1 + 1, generator=g, dtype=torch.float64), -1).values
    w1 = (torch.rand(N, T1, generator=g, dtype=torch.float64) * 0.05).requires_grad_(True)
    loss = proposal_loss([t1, t_ref], [w1, w_ref])
    loss.backward()
    ours = np.zeros((N, T1))
    val = 0.0
    c_prop = 1.0 / (N * T0)
    for r in range(N):
        cw = np.concatenate([[0.0], np.cumsum(w1.detach().numpy()[r])])
        dd = np.zeros(T1 + 1)
        for i in range(T0):
            lo = _upper_bound(t1[r, :-1].numpy(), t_ref[r, i].item()) - 1
            hi = _upper_bound(t1[r, 1:].numpy(), t_ref[r, i + 1].item())
            lo, hi = min(max(lo, 0), T1 - 1), min(max(hi, 0), T1 - 1)
            x = w_ref[r, i].item() - (cw[hi + 1] - cw[lo])
            if x > 0:
                den = w_ref[r, i].item() + 1e-8
                val += x * x / den
                gr = -2 * x / den * c_prop
                dd[lo] += gr
                dd[hi + 1] -= gr
        ours[r] = np.cumsum(dd)[:T1]
    assert abs(val * c_prop - loss.item()) <= 1e-12 * max(1.0, abs(loss.item()))
    np.testing.assert_allclose(ours, w1.grad.numpy(), rtol=1e-9, atol=1e-14)
    assert (np.abs(ours) > 0).any()
