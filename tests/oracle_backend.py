"""Test infrastructure: `_gridencoder` / `_shencoder`-compatible backends on
the C oracle (oracle/encoders_oracle.c), for CPU tensors.

Swapping them into the mirror modules (gridencoder.grid._backend,
shencoder.sphere_harmonics._backend) gives a CPU twin of the product's
unfused path whose autograd graph is the same torch ops with the oracle's
encoder forward/backward -- the reference's own structure -- so GPU gradients
of a training step can be compared against it.  Never used by the product.
"""
import contextlib

import numpy as np
import torch

from oracle import encoders as enc


class GridBackend:
    @staticmethod
    def grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, max_level, S, H,
                            dy_dx, gridtype, align_corners, interpolation):
        assert dy_dx is None and gridtype == 0 and not align_corners and interpolation == 0
        out = enc.grid_encode_forward(inputs.detach().numpy(), embeddings.detach().numpy(),
                                      offsets.numpy(), L, S, H, max_level=max_level)
        outputs.copy_(torch.from_numpy(np.ascontiguousarray(out)))

    @staticmethod
    def grid_encode_backward(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L,
                             max_level, S, H, dy_dx, grad_inputs, gridtype, align_corners,
                             interpolation):
        assert dy_dx is None and grad_inputs is None
        g = enc.grid_encode_backward(grad.detach().numpy(), inputs.detach().numpy(),
                                     embeddings.detach().numpy(), offsets.numpy(), L, S, H,
                                     max_level=max_level)
        grad_embeddings.copy_(torch.from_numpy(np.ascontiguousarray(g)))


class SHBackend:
    @staticmethod
    def sh_encode_forward(inputs, outputs, B, input_dim, degree, dy_dx):
        assert dy_dx is None
        out = enc.sh_encode_forward(inputs.detach().numpy(), degree)
        out = out[0] if isinstance(out, tuple) else out
        outputs.copy_(torch.from_numpy(np.ascontiguousarray(out)))


class _RecordingGridBackend(GridBackend):
    """GridBackend that also keeps every forward call's inputs (fp32, in call
    order): the sample positions the fp32 computation encoded."""
    store = None

    @classmethod
    def grid_encode_forward(cls, inputs, *args):
        cls.store.append(inputs.detach().clone())
        GridBackend.grid_encode_forward(inputs, *args)


@contextlib.contextmanager
def oracle_encoders(record=None):
    """Route the mirror's GridEncoder / SHEncoder through the C oracle.
    record: a list that receives every grid-encoder call's inputs."""
    import gridencoder.grid as g
    import shencoder.sphere_harmonics as s
    old = (g._backend, s._backend)
    gb = GridBackend
    if record is not None:
        gb = type("_Rec", (_RecordingGridBackend,), {"store": record})
    g._backend, s._backend = gb, SHBackend
    try:
        yield
    finally:
        g._backend, s._backend = old


# --------------------------------------------------------- float64 twin --
# The reference's op sequence with every operation in float64: the encoders
# as differentiable torch ops (the same corner rows as gridencoder.cu:45-79 and
# the same SH polynomials as shencoder.cu:43-68, evaluated in double), and
# trunc_exp without the fp32 cast of its custom_fwd.  Used as the "exact"
# gradient against which the fp32 computations (HIP kernels, fp32 CPU twin)
# are measured.

_P1, _P2 = 2654435761, 805459861


_REPLAY = []


def _grid_encode64(inputs, embeddings, offsets, per_level_scale, base_resolution,
                   calc_grad_inputs=False, gridtype=0, align_corners=False, interpolation=0,
                   max_level=None):
    """float64 grid encoding at the fp32 computation's own interpolation
    coordinates: the inputs are replaced by the recorded fp32 inputs of the
    same call (float64_twin(grid_inputs=...)), and the cell / fraction come
    from the reference's fp32 position fmaf(u, res, -0.5) (gridencoder.cu:148);
    the corner weights and the weighted sums are float64.  A 1-ulp change of u
    moves the finest level's fraction by ~5e-4, so the "exact" gradient is the
    one at the sample positions the fp32 paths share (bit-identical between the
    HIP kernels and the fp32 twin)."""
    assert gridtype == 0 and not align_corners and interpolation == 0
    u = inputs.double()
    if _REPLAY:
        rec = _REPLAY.pop(0)
        assert rec.shape == inputs.shape, (rec.shape, inputs.shape)
        drift = (rec.double() - u).abs().max().item() if rec.numel() else 0.0
        assert drift < 1e-5, f"float64 twin: sample positions drifted from the fp32 run by {drift}"
        u = rec.double()
    offs = [int(v) for v in offsets.cpu().tolist()]
    L = len(offs) - 1
    ml = L if max_level is None else min(max_level, L)
    S = float(np.log2(per_level_scale))
    res_l = enc.grid_level_resolutions(L, S, int(base_resolution))
    outside = ((u < 0) | (u > 1)).any(-1, keepdim=True)          # kernel_grid: such points -> 0
    outs = []
    for lvl in range(L):
        C = embeddings.shape[1]
        if lvl >= ml:
            outs.append(torch.zeros(u.shape[0], C, dtype=embeddings.dtype))
            continue
        size, res = offs[lvl + 1] - offs[lvl], res_l[lvl]
        # fmaf(u, res, -0.5) in fp32: u * res is exact in double (24 x 13
        # bits) and so is the -0.5, so one rounding to fp32 reproduces it
        pos = (u * res - 0.5).float().double().clamp(0, res - 1)
        cell = torch.floor(pos)
        frac = pos - cell
        cell = cell.long()
        hashed = res ** 3 > size
        acc = 0
        for c in range(8):
            w = 1
            idx = []
            for d in range(3):
                if (c >> d) & 1:
                    w = w * frac[:, d]
                    idx.append(torch.clamp(cell[:, d] + 1, max=res - 1))
                else:
                    w = w * (1 - frac[:, d])
                    idx.append(cell[:, d])
            if hashed:
                row = idx[0] ^ ((idx[1] * _P1) & 0xFFFFFFFF) ^ ((idx[2] * _P2) & 0xFFFFFFFF)
            else:
                row = idx[0] + idx[1] * res + idx[2] * res * res
            row = row % size
            acc = acc + w[:, None] * embeddings[offs[lvl] + row]
        outs.append(torch.where(outside, torch.zeros((), dtype=embeddings.dtype), acc))
    return torch.cat(outs, dim=1)


def _sh_encode64(inputs, degree, calc_grad_inputs=False):
    assert degree == 4
    x, y, z = inputs.double().unbind(-1)
    x2, y2, z2 = x * x, y * y, z * z
    xy, yz, xz = x * y, y * z, x * z
    return torch.stack([
        torch.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
        -0.48860251190291987 * x, 1.0925484305920792 * xy, -1.0925484305920792 * yz,
        0.94617469575755997 * z2 - 0.31539156525251999, -1.0925484305920792 * xz,
        0.54627421529603959 * x2 - 0.54627421529603959 * y2,
        0.59004358992664352 * y * (-3.0 * x2 + y2), 2.8906114426405538 * xy * z,
        0.45704579946446572 * y * (1.0 - 5.0 * z2), 0.3731763325901154 * z * (5.0 * z2 - 3.0),
        0.45704579946446572 * x * (1.0 - 5.0 * z2), 1.4453057213202769 * z * (x2 - y2),
        0.59004358992664352 * x * (-x2 + 3.0 * y2)], dim=-1)


class _TruncExp64(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * torch.exp(x.clamp(-15, 15))


@contextlib.contextmanager
def float64_twin(grid_inputs=None):
    """Route the mirror's encoders and trunc_exp through float64 torch ops and
    make float64 the default dtype (the renderer's linspaces), for a network
    converted with .double() on the CPU.  grid_inputs: the fp32 run's recorded
    encoder inputs (oracle_encoders(record=...)), used in place of the float64
    run's own sample positions, call by call."""
    import gridencoder.grid as g
    import nerf.network as nw
    import shencoder.sphere_harmonics as s
    old = (g.grid_encode, s.sh_encode, nw.trunc_exp, torch.get_default_dtype())
    g.grid_encode, s.sh_encode, nw.trunc_exp = _grid_encode64, _sh_encode64, _TruncExp64.apply
    torch.set_default_dtype(torch.float64)
    _REPLAY[:] = list(grid_inputs or [])
    try:
        yield
        assert not _REPLAY, f"float64 twin: {len(_REPLAY)} recorded encoder calls not replayed"
    finally:
        _REPLAY[:] = []
        g.grid_encode, s.sh_encode, nw.trunc_exp = old[:3]
        torch.set_default_dtype(old[3])


@contextlib.contextmanager
def injected_bins(bins):
    """The renderer's resampled bins (sample_pdf's outputs of the proposal
    stages, in call order) replaced by the given tensors -- e.g. those the HIP
    kernels computed (FusedRenderer.render(taps=True)) -- so that a CPU twin
    evaluates the step at the HIP path's own sample positions.  The injected
    bins must agree with what the twin computes to 1e-5 (a different pdf
    walk would not be the same step)."""
    import nerf.renderer as rr
    old = rr.sample_pdf
    queue = list(bins)

    def fake(b, w, T, perturb=False):
        mine = old(b, w, T, perturb)
        inj = queue.pop(0).to(dtype=mine.dtype, device=mine.device).contiguous()
        assert inj.shape == mine.shape, (inj.shape, mine.shape)
        drift = (inj - mine).abs().max().item()
        assert drift < 1e-5, f"injected bins differ from the twin's by {drift}"
        return inj
    rr.sample_pdf = fake
    try:
        yield
        assert not queue, f"{len(queue)} injected bins not used"
    finally:
        rr.sample_pdf = old


@contextlib.contextmanager
def recorded_bins(store):
    """Keep the renderer's resampled bins (sample_pdf outputs, call order) in
    `store` -- to inject them into another run (injected_bins)."""
    import nerf.renderer as rr
    old = rr.sample_pdf

    def rec(*a, **k):
        out = old(*a, **k)
        store.append(out.detach().clone())
        return out
    rr.sample_pdf = rec
    try:
        yield store
    finally:
        rr.sample_pdf = old
