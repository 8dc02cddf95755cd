"""Fused ray-march render on gfx950 (samnerf_render_forward, raymarch.hip).

`FusedRenderer(net)` wraps a NeRFNetwork-shaped module (the mirror in
nerf/network.py, or anything exposing the same attributes / state_dict keys)
and renders rays with the whole NeRFRenderer.run loop
(nerf/renderer.py:221-390) in five kernel launches.  Parameters are read in
place (torch layout); nothing is copied or cached between calls except the
workspace buffer.
"""
import ctypes

import numpy as np
import torch

from ._lib import SamnerfGrid, SamnerfModel, SamnerfRgbGrads, SamnerfTaps, check, lib
from .ops import _ptr, _stream

ROW = 164          # head-input row: f_sam 128 | f_image 31 | image 3 | depth 1 | pad


def _param(t, name):
    if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
        raise RuntimeError(f"fused render: {name} must be a contiguous float32 CUDA tensor")
    return ctypes.c_void_p(t.data_ptr())


def mask_kind(net):
    """The fused kernels' mask_kind for the network's --with_mask head, or None
    when it runs on the unfused path: 0 'default' (K <= 32), 1 'adaptive' /
    'density', 2 'adaptive' / 'rgb' with sum_after_mlp (without it the
    reference's view_mlp intermediates are per ray and its cat fails); the
    'lightweight_mask' and adaptive 'sam' heads raise in the reference."""
    o = net.opt
    if not getattr(o, "with_mask", False):
        return None
    if o.mask_mlp_type == "default":
        return 0 if net.mask_mlp[0].net[2].weight.shape[0] <= 32 else None
    if o.mask_mlp_type == "adaptive" and net.mask_mlp[-1].weight.shape[0] <= 32:
        if o.adaptive_mlp_type == "density":
            return 1
        if o.adaptive_mlp_type == "rgb" and getattr(o, "sum_after_mlp", False):
            return 2
    return None


def perturbed_positions(N, num_steps, device):
    """The sample positions of perturb=True, drawn and computed exactly as the
    reference does (torch.rand_like in its order, the same expressions): the
    stage-0 bins (renderer.py:264-271) and sample_pdf's u for stages 1 and 2
    (renderer.py:97-103, called at :274-275).  The proposal stages draw nothing
    else, so drawing all three first consumes the generator identically.
    Returns (bins0 [N, T0+1], u1 [N, T1+1], u2 [N, T2+1])."""
    T0 = int(num_steps[0])
    bins = torch.linspace(0, 1, T0 + 1, device=device).unsqueeze(0).expand(N, -1)
    bins = (bins + (torch.rand_like(bins) - 0.5) / T0).clamp(0, 1)
    out = [bins.contiguous()]
    for T in (int(num_steps[1]) + 1, int(num_steps[2]) + 1):
        u = torch.linspace(0.5 / T, 1 - 0.5 / T, steps=T).to(device).expand(N, T)   # on the CPU, then moved, as renderer.py:97
        u = u + (torch.rand_like(u) - 0.5) / T
        out.append(u.contiguous())
    return tuple(out)


def ray_of_slots(N, view_width):
    """The kernels' slot -> ray map (samnerf_common.h RayTiles / make_ray_tiles):
    with a view width W (a multiple of 8, N a multiple of 4 W rows) slot s is
    pixel (x, y) of 8 x 4 tile s // 32 in row-major tile order, pixel s % 32
    row-major inside it; the identity otherwise.  int64 [N] (CPU)."""
    s = torch.arange(N, dtype=torch.int64)
    W = int(view_width)
    if W < 8 or W % 8 or N % (4 * W):
        return s
    tile, inn = s >> 5, s & 31
    trow, tcol = tile // (W // 8), tile % (W // 8)
    return (trow * 4 + (inn >> 3)) * W + tcol * 8 + (inn & 7)


def last_forms():
    """The compiled kernel forms the calling thread's last render launched
    (samnerf_last_forms): [prop0 level classes, prop1 level classes, k_final
    layout, 0]; level classes = dense mask | hashed mask << 8, 0 = run-time."""
    out = (ctypes.c_uint32 * 4)()
    lib().samnerf_last_forms(out, 4)
    return list(out)


class FusedRenderer:
    """head_mode: 0 = f16x3 (each fp32 product of grid_mlp, the SAM head and
    the mask head as three fp16 MFMA products on power-of-two scaled operands:
    fp32-equivalent, csrc/f16x3.h; default), 1 = exact fp32 MFMA.  t_thresh: 0 (default) = the reference's
    semantics; > 0 = the flagged non-parity early-exit mode N1 (a wave stops
    marching once every ray's transmittance is below t_thresh; include/
    samnerf_hip.h).  Unset, both follow the network's head_mode / t_thresh
    attributes (NeRFRenderer, defaults 0)."""

    def __init__(self, net, head_mode=None, t_thresh=None, deterministic=False):
        """deterministic=True: the s_grid gradient of the distillation step
        (sgrid_backward) sums in 64-bit fixed point (samnerf_sgrid_backward_det,
        SURVEY H5) so identical steps give identical bits; the default is the
        reference's unordered fp32 atomics."""
        self.net = net
        self.deterministic = bool(deterministic)
        self._accum = None
        self._ws = None
        self._packed = {}      # (device, stream) -> what its workspace's packed weights are
        self.last_reuse_packed = 0
        self._keep = []
        self._model = None
        self._model_key_cached = None
        self._head_mode = head_mode
        self._t_thresh = None if t_thresh is None else float(t_thresh)
        if not 0.0 <= self.t_thresh < 1.0:
            raise ValueError(f"t_thresh {self.t_thresh} outside [0, 1)")

    # explicit arguments win; otherwise the network's attributes (NeRFRenderer.
    # head_mode / t_thresh, defaults 0): no environment variable changes the path
    @property
    def head_mode(self):
        return int(self._head_mode if self._head_mode is not None else getattr(self.net, "head_mode", 0))

    @property
    def t_thresh(self):
        return float(self._t_thresh if self._t_thresh is not None else getattr(self.net, "t_thresh", 0.0))

    # --------------------------------------------------------------- model --
    def _grid(self, enc, name):
        offs = np.ascontiguousarray(enc.offsets_host, np.int32)
        self._keep.append(offs)
        g = SamnerfGrid()
        g.embeddings = _param(enc.embeddings, name + ".embeddings")
        g.offsets_host = offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        g.num_levels = enc.num_levels
        g.level_dim = enc.level_dim
        g.S = float(np.log2(enc.per_level_scale))
        g.base_resolution = enc.base_resolution
        return g

    def _model_key(self):
        """What the samnerf_model struct depends on: parameter addresses (the
        struct holds pointers, values may change freely, e.g. under Adam) and
        the by-value fields (aabb, bounds, steps)."""
        n = self.net
        aabb = n.aabb_train if n.training else n.aabb_infer
        return (n.training, self.head_mode, self.t_thresh, aabb.data_ptr(), aabb._version,
                tuple(p.data_ptr() for p in n.parameters()), tuple(n.opt.num_steps),
                float(n.opt.min_near), float(n.bound), bool(n.opt.with_sam))

    def model(self):
        """The samnerf_model struct of the wrapped network, rebuilt only when
        _model_key changes: reading the aabb back to the host would otherwise
        synchronise the stream on every call and stall the launch queue."""
        key = self._model_key()
        if self._model is not None and key == self._model_key_cached:
            return self._model
        self._model = self._build_model()
        self._model_key_cached = key
        return self._model

    def _build_model(self):
        n = self.net
        opt = n.opt
        self._keep = []
        m = SamnerfModel()
        m.grid = self._grid(n.grid, "grid")
        m.prop[0] = self._grid(n.prop_encoders[0], "prop_encoders.0")
        m.prop[1] = self._grid(n.prop_encoders[1], "prop_encoders.1")
        for i in range(3):
            m.grid_mlp[i] = _param(n.grid_mlp.net[i].weight, f"grid_mlp.net.{i}.weight")
            m.view_mlp[i] = _param(n.view_mlp.net[i].weight, f"view_mlp.net.{i}.weight")
        for p in range(2):
            for i in range(2):
                m.prop_mlp[p][i] = _param(n.prop_mlp[p].net[i].weight, f"prop_mlp.{p}.net.{i}.weight")
        m.with_sam = int(bool(opt.with_sam))
        if opt.with_sam:
            m.s_grid = self._grid(n.s_grid, "s_grid")
            skip = n.samvit_mlp[0]
            for i in range(5):
                m.sam_w[i] = _param(skip.net[i].weight, f"samvit_mlp.0.net.{i}.weight")
                m.sam_b[i] = _param(skip.net[i].bias, f"samvit_mlp.0.net.{i}.bias")
            m.ln_w = _param(n.samvit_mlp[1].weight, "samvit_mlp.1.weight")
            m.ln_b = _param(n.samvit_mlp[1].bias, "samvit_mlp.1.bias")
        aabb = n.aabb_train if n.training else n.aabb_infer
        for i, v in enumerate(aabb.detach().cpu().tolist()):
            m.aabb[i] = v
        m.grid_bound = float(n.bound)
        m.min_near = float(opt.min_near)
        for i, v in enumerate(opt.num_steps):
            m.num_steps[i] = int(v)
        m.head_mode = int(self.head_mode)
        m.t_thresh = float(self.t_thresh)
        kind = mask_kind(n)
        if kind == 0:                                   # --with_mask, mask_mlp_type 'default'
            m.m_grid = self._grid(n.m_grid, "m_grid")
            skip = n.mask_mlp[0]
            for i in range(3):
                m.mask_w[i] = _param(skip.net[i].weight, f"mask_mlp.0.net.{i}.weight")
            m.mask_out = int(skip.net[2].weight.shape[0])
        elif kind is not None:                          # 'adaptive': density / rgb
            for i, lin in enumerate(n.mask_mlp):
                m.mask_w[i] = _param(lin.weight, f"mask_mlp.{i}.weight")
            m.mask_out = int(n.mask_mlp[-1].weight.shape[0])
        m.mask_kind = kind or 0
        m.with_mask = 0                                 # set per call (render(mask=True))
        m.sum_after_mlp = int(bool(getattr(opt, "sum_after_mlp", False)))
        return m

    def invalidate_packed(self):
        """Forget the packed weights of every workspace: call after changing
        grid_mlp or SAM-head weights in a way torch's version counter does not
        see (writes through `.data`, or through raw pointers from C)."""
        self._packed = {}

    def _pack_signature(self, m):
        """What the packed weights of a render depend on: head_mode and the
        packed tensors (grid_mlp, the SAM head's weights) as (data pointer,
        torch version counter) -- an in-place update (optimizer step, copy_,
        load_state_dict, FusedAdam) bumps the counter, a new tensor changes
        the pointer; `.data` writes do not (invalidate_packed)."""
        n = self.net
        ts = [n.grid_mlp.net[i].weight for i in range(3)]
        if m.with_sam:
            ts += [n.samvit_mlp[0].net[i].weight for i in range(5)]
        # (the packed regions lead the workspace, raymarch.hip carve(): their
        # place does not depend on N; the model fields before them are here)
        return (int(m.head_mode), int(m.with_sam), tuple((t.data_ptr(), t._version) for t in ts))

    def workspace(self, m, N, device):
        """Scratch of one render call, one buffer per (device, stream): calls
        on one stream reuse it in stream order; renders issued on different
        streams (concurrent views) never share one."""
        need = lib().samnerf_render_workspace_size(ctypes.byref(m), N)
        key = (device, _stream_key(device))
        if self._ws is None:
            self._ws = {}
        ws = self._ws.get(key)
        if ws is None or ws.numel() < need:
            ws = self._ws[key] = torch.empty(max(need, 1), dtype=torch.uint8, device=device)
        return ws, need

    def fused_mask_ok(self):
        """The network's mask head runs on the fused kernels (mask_kind)."""
        return mask_kind(self.net) is not None

    # -------------------------------------------------------------- render --
    @torch.no_grad()
    def render(self, rays_o, rays_d, cam_near_far=None, bg_color=None, rows=None,
               keep_workspace=False, feats=True, taps=False, own_workspace=False, view_width=0,
               mask=False, perturb=False, mask_logits=True, out_tile=None):
        """rays_o, rays_d [N,3] (CUDA fp32) -> dict(image [N,3], depth [N],
        weights_sum [N], samvit [N,256] if with_sam and feats).  `rows`
        (optional [N,164] tensor) receives the head input cat(f_sam, f_image,
        image, depth).  feats=False skips the SAM-feature stages (the
        reference computes and discards them when return_feats == 0).
        taps=True (parity tests) adds the stages' intermediates
        (samnerf_set_taps): ds0 [N,128], ds1 [N,64], their weights w0, w1, bins1 [N,65],
        bins2 [N,33] and their searchsorted indices inds1, inds2 (int32), the
        final stage's sigma2, w2 [N,32] and positions u2 [N,32,3] -- ray-major
        views of the kernels' sample-major buffers -- and the corner rows
        rows2 (grid, k_final) and srows (s_grid, k_sgrid_box4; -1 where a
        sample was skipped) [len(tap_rays), 32, 16, 8] int32 (level-relative)
        of every stride-th kernel SLOT (slots 0, stride, 2 stride, ..).
        tap_rays holds the ray ids of those slots, in the rows' order:
        without view_width it is arange(0, N, stride); with view_width
        (ray tiles) it is ray_of_slots(N, view_width)[arange(0, N, stride)],
        neither sorted nor evenly spaced -- pair rows2[i] / srows[i] with
        tap_rays[i], never with i * stride.  taps=<int> sets the stride
        (default 61).
        own_workspace=True renders into a fresh workspace (from torch's
        caching allocator) instead of the per-stream one, so a caller can
        keep it (training: the backward reads its sample weights/positions).
        view_width: the rays are a row-major image of this width (a layout
        hint, samnerf_model.view_width): the kernels then run 8 x 4 pixel
        tiles per wave, same outputs bit for bit, faster gathers.
        mask=True (a 'default' mask head, fused_mask_ok): also
        instance_mask_logits [N, n_inst + redundant_instance]
        (samnerf_mask_forward on the render's workspace); with
        mask_logits=False the samples' geo_feat are stored for a later
        samnerf_mask_train_forward and no logits are computed.
        out_tile: a contiguous fp32 CUDA tensor [N, C] (C >= 261 with SAM
        features, >= 5 without): the outputs are written into its rows --
        columns 0-2 image, 3 depth, 4 weights_sum, 5-260 samvit
        (samnerf_render_forward_tile; the all-gather record of a sharded view)
        -- and returned as views of it.
        perturb: False (default), True (draw the perturbed sample positions
        with torch's generator, perturbed_positions -- the reference's
        perturb=True), or a (bins0, u1, u2) tuple of them [N, 129], [N, 65],
        [N, 33] (samnerf_model.perturb)."""
        rays_o = rays_o.contiguous().float()
        rays_d = rays_d.contiguous().float()
        N = rays_o.shape[0]
        dev = rays_o.device
        m = self.model()
        m.view_width = int(view_width or 0)
        if mask and not self.fused_mask_ok():
            raise NotImplementedError("fused render: this mask head runs on the unfused path")
        # 2: a training render (mask_logits=False): the adaptive heads keep their per-ray input sums
        m.with_mask = (2 if not mask_logits else 1) if mask else 0
        pert = None
        if isinstance(perturb, (tuple, list)) or perturb:      # the GUI passes spp (an int) as perturb
            pert = tuple(perturb) if isinstance(perturb, (tuple, list)) else \
                perturbed_positions(N, list(m.num_steps), dev)
            shapes = [(N, int(m.num_steps[0]) + 1), (N, int(m.num_steps[1]) + 1), (N, int(m.num_steps[2]) + 1)]
            if len(pert) != 3 or any(tuple(t.shape) != sh for t, sh in zip(pert, shapes)):
                raise ValueError(f"fused render: perturb arrays must have shapes {shapes}")
            pert = tuple(t.contiguous().float() for t in pert)
            for i in range(3):
                m.perturb[i] = _param(pert[i], f"perturb[{i}]")
        else:
            for i in range(3):
                m.perturb[i] = None
        pack_key = None
        if own_workspace:
            need = lib().samnerf_render_workspace_size(ctypes.byref(m), N)
            ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
            m.reuse_packed = 0
        else:
            ws, need = self.workspace(m, N, dev)
            # the packed MLP weights this per-stream workspace holds from its
            # last render are reused when the weights are the same tensors at
            # the same version (samnerf_model.reuse_packed: ~25 us per view);
            # the SAM head's are packed only by renders that run the head
            head = bool(m.with_sam and feats)
            pack_key = (ws.data_ptr(), self._pack_signature(m))
            have = self._packed.get((dev, _stream_key(dev)))
            m.reuse_packed = int(have is not None and have[0] == pack_key and (have[1] or not head))
        if bg_color is None:
            bg = 1.0
        elif torch.is_tensor(bg_color):
            if bg_color.numel() != 1:
                raise NotImplementedError("fused render: per-ray background colours")
            bg = float(bg_color)
        else:
            bg = float(bg_color)
        if out_tile is not None:
            need_c = 261 if (m.with_sam and feats) else 5
            if (out_tile.dim() != 2 or out_tile.shape[0] != N or out_tile.shape[1] < need_c
                    or out_tile.dtype != torch.float32 or not out_tile.is_contiguous()
                    or out_tile.device != dev):
                raise ValueError(f"fused render: out_tile must be a contiguous fp32 [{N}, >={need_c}] "
                                 f"tensor on {dev}")
            if mask:
                raise NotImplementedError("fused render: out_tile with mask outputs")
            image, depth, wsum = out_tile[:, 0:3], out_tile[:, 3], out_tile[:, 4]
            samvit = out_tile[:, 5:261] if need_c == 261 else None
        else:
            image = torch.empty(N, 3, device=dev)
            depth = torch.empty(N, device=dev)
            wsum = torch.empty(N, device=dev)
            samvit = torch.empty(N, 256, device=dev) if (m.with_sam and feats) else None
        cnf = None
        n_cnf = 0
        if cam_near_far is not None:
            cnf = cam_near_far.contiguous().float()
            n_cnf = cnf.shape[0]
        if rows is not None:
            assert rows.shape == (N, ROW) and rows.is_contiguous()
        tap = None
        if taps:
            steps = [int(v) for v in m.num_steps]
            stride = 61 if taps is True else int(taps)
            n_tap = (N + stride - 1) // stride
            tap = {"ds0": torch.empty(steps[0], N, device=dev), "ds1": torch.empty(steps[1], N, device=dev),
                   "w0": torch.empty(steps[0], N, device=dev), "w1": torch.empty(steps[1], N, device=dev),
                   "bins1": torch.empty(steps[1] + 1, N, device=dev),
                   "bins2": torch.empty(steps[2] + 1, N, device=dev),
                   "inds1": torch.empty(steps[1] + 1, N, device=dev, dtype=torch.int32),
                   "inds2": torch.empty(steps[2] + 1, N, device=dev, dtype=torch.int32),
                   "sigma2": torch.empty(steps[2], N, device=dev), "w2": torch.empty(steps[2], N, device=dev),
                   "u2": torch.empty(steps[2], 3, N, device=dev)}
            rows_tap = {"rows2": torch.full((n_tap, steps[2], 16, 8), -1, device=dev, dtype=torch.int32),
                        "srows": torch.full((n_tap, steps[2], 16, 8), -1, device=dev, dtype=torch.int32)}
            st = SamnerfTaps(*[t.data_ptr() for t in tap.values()], stride,
                             rows_tap["rows2"].data_ptr(), rows_tap["srows"].data_ptr())
            check(lib().samnerf_set_taps(ctypes.byref(st), N), "set_taps")
        try:
            if out_tile is not None:
                check(lib().samnerf_render_forward_tile(
                    ctypes.byref(m), _ptr(rays_o), _ptr(rays_d), N, _ptr(cnf), n_cnf, bg, _ptr(out_tile),
                    out_tile.shape[1], int(samvit is not None), _ptr(rows), _ptr(ws), need, _stream(rays_o)),
                    "render_forward_tile")
            else:
                check(lib().samnerf_render_forward(
                    ctypes.byref(m), _ptr(rays_o), _ptr(rays_d), N, _ptr(cnf), n_cnf, bg, _ptr(image),
                    _ptr(depth), _ptr(wsum), _ptr(samvit), _ptr(rows), _ptr(ws), need, _stream(rays_o)),
                    "render_forward")
            self.last_reuse_packed = int(m.reuse_packed)
            if pack_key is not None:
                key = (dev, _stream_key(dev))
                if m.reuse_packed:                 # nothing packed: the head's stays as it was
                    head = head or self._packed[key][1]
                self._packed[key] = (pack_key, head)
            if mask and mask_logits:
                logits = torch.empty(N, int(m.mask_out), device=dev)
                check(lib().samnerf_mask_forward(ctypes.byref(m), N, _ptr(logits), _ptr(ws), need,
                                                 _stream(rays_o)), "mask_forward")
        finally:
            if taps:
                lib().samnerf_set_taps(None, 0)
            for i in range(3):
                m.perturb[i] = None
            m.reuse_packed = 0
        out = {"image": image, "depth": depth, "weights_sum": wsum}
        if mask and mask_logits:
            out["instance_mask_logits"] = logits
        if tap is not None:
            # the kernels keep per-sample intermediates in slot order (ray
            # tiling, samnerf_model.view_width): back to ray order here
            ray_of = ray_of_slots(N, int(m.view_width)).to(dev)
            u2 = tap.pop("u2")
            for k, v in tap.items():
                r = torch.empty_like(v.t())
                r[ray_of] = v.t()
                out[k] = r
            r = torch.empty_like(u2.permute(2, 0, 1))
            r[ray_of] = u2.permute(2, 0, 1)
            out["u2"] = r
            out.update(rows_tap)
            out["tap_rays"] = ray_of[torch.arange(0, N, stride, device=dev)].cpu()
        if samvit is not None:
            out["samvit"] = samvit
        if keep_workspace:
            out["_workspace"] = (ws, need, m, int(m.view_width))
        return out

    @torch.no_grad()
    def sam_head(self, rows):
        """samvit_mlp (SkipConnMLP + LayerNorm, network.py:36-75, :120-123) on
        head-input rows [N,164] (render(rows=...)'s layout) at this renderer's
        head_mode -> samvit [N,256] (samnerf_sam_head_forward)."""
        rows = rows.contiguous().float()
        assert rows.dim() == 2 and rows.shape[1] == ROW, rows.shape
        N = rows.shape[0]
        m = self.model()
        need = lib().samnerf_sam_head_workspace_size()
        ws = torch.empty(need, dtype=torch.uint8, device=rows.device)
        out = torch.empty(N, 256, device=rows.device)
        check(lib().samnerf_sam_head_forward(ctypes.byref(m), _ptr(rows), N, _ptr(out), _ptr(ws), need,
                                             _stream(rows)), "sam_head_forward")
        return out

    def sgrid_backward(self, grad_rows, workspace, grad_embeddings):
        ws, need, m, view_width = workspace
        m.view_width = view_width                 # the forward's slot order of the workspace
        N = grad_rows.shape[0]
        grad_rows = grad_rows.contiguous()
        assert grad_rows.shape[1] == ROW
        if self.deterministic:
            # one fixed-point accumulator per (device, stream), like workspace():
            # calls on one stream reuse it in order (each leaves it zero);
            # concurrent calls on other streams never share one
            size = lib().samnerf_sgrid_accum_size(ctypes.byref(m))
            dev = grad_rows.device
            key = (dev, torch.cuda.current_stream(dev).cuda_stream)
            if self._accum is None:
                self._accum = {}
            acc = self._accum.get(key)
            if acc is None or acc.numel() < size:
                acc = self._accum[key] = torch.zeros(max(size, 1), dtype=torch.uint8, device=dev)
            check(lib().samnerf_sgrid_backward_det(ctypes.byref(m), _ptr(grad_rows), N,
                                                   _ptr(grad_embeddings), _ptr(acc), acc.numel(), _ptr(ws),
                                                   need, _stream(grad_rows)), "sgrid_backward_det")
            return
        check(lib().samnerf_sgrid_backward(ctypes.byref(m), _ptr(grad_rows), N,
                                           _ptr(grad_embeddings), _ptr(ws), need,
                                           _stream(grad_rows)), "sgrid_backward")


def _stream_key(device):
    return torch.cuda.current_stream(device).cuda_stream


class _FusedSamRows(torch.autograd.Function):
    """Head-input rows with gradient w.r.t. s_grid.embeddings only (RGB params
    are frozen in the distillation stage, main.py:255-262; proposal grads are
    cut by sample_pdf(...).detach(), renderer.py:274-275)."""

    @staticmethod
    def forward(ctx, s_emb, renderer, rays_o, rays_d, cam_near_far, bg_color, view_width):
        N = rays_o.shape[0]
        rows = torch.empty(N, ROW, device=rays_o.device)
        # feats=False: the head runs in torch below (it needs autograd), so the
        # fused head is skipped; a private workspace keeps the sample weights
        # and positions the s_grid scatter of the backward reads
        out = renderer.render(rays_o, rays_d, cam_near_far, bg_color, rows=rows,
                              keep_workspace=True, feats=False, own_workspace=True,
                              view_width=view_width)
        ctx.ws = out.pop("_workspace")
        ctx.renderer = renderer
        ctx.keep = list(renderer._keep)
        ctx.emb_shape = s_emb.shape
        ctx.mark_non_differentiable(out["image"], out["depth"], out["weights_sum"])
        return rows, out["image"], out["depth"], out["weights_sum"]

    @staticmethod
    def backward(ctx, g_rows, g_img, g_depth, g_wsum):
        grad = None
        if ctx.needs_input_grad[0] and g_rows is not None:
            grad = torch.zeros(ctx.emb_shape, device=g_rows.device)
            ctx.renderer.sgrid_backward(g_rows, ctx.ws, grad)
        return grad, None, None, None, None, None, None


def _head_params(net):
    skip, ln = net.samvit_mlp[0], net.samvit_mlp[1]
    return ([skip.net[i].weight for i in range(5)] + [skip.net[i].bias for i in range(5)]
            + [ln.weight, ln.bias])


class _SamHeadTrain(torch.autograd.Function):
    """samvit_mlp (SkipConnMLP 163->256 x5 + LayerNorm, network.py:36-75,
    :120-123) on the head-input rows, forward and backward as HIP kernels
    (sam_head_train.hip, exact fp32 MFMA): gradients w.r.t. the rows and the
    12 head tensors, the same values torch's autograd computes for
    net.samvit_mlp(rows[:, :163]) up to summation order."""

    @staticmethod
    def forward(ctx, rows, renderer, *params):
        rows = rows.contiguous()
        N = rows.shape[0]
        m = renderer.model()
        need = lib().samnerf_head_train_workspace_size(N)
        ws = torch.empty(max(need, 1), dtype=torch.uint8, device=rows.device)
        samvit = torch.empty(N, 256, device=rows.device)
        check(lib().samnerf_head_train_forward(ctypes.byref(m), _ptr(rows), N, _ptr(samvit), _ptr(ws),
                                               need, _stream(rows)), "head_train_forward")
        ctx.save_for_backward(rows)
        ctx.ws, ctx.need, ctx.m, ctx.keep = ws, need, m, list(renderer._keep)
        ctx.shapes = [p.shape for p in params]
        return samvit

    @staticmethod
    def backward(ctx, g):
        (rows,) = ctx.saved_tensors
        g = g.contiguous().float()
        dev = rows.device
        grows = torch.empty_like(rows)                     # all written by the kernels
        grads = [torch.empty(sh, device=dev) for sh in ctx.shapes]
        gw = (ctypes.c_void_p * 5)(*[t.data_ptr() for t in grads[:5]])
        gb = (ctypes.c_void_p * 5)(*[t.data_ptr() for t in grads[5:10]])
        check(lib().samnerf_head_train_backward(
            ctypes.byref(ctx.m), _ptr(rows), _ptr(g), rows.shape[0], _ptr(grows), gw, gb,
            _ptr(grads[10]), _ptr(grads[11]), _ptr(ctx.ws), ctx.need, _stream(g)), "head_train_backward")
        return (grows, None, *grads)


def render_sam_train(renderer, rays_o, rays_d, cam_near_far=None, bg_color=None, head=None,
                     view_width=0):
    """Differentiable SAM-feature render for the distillation step
    (nerf/utils.py:1098-1099): returns samvit [N,256] with autograd to
    s_grid.embeddings (HIP scatter) and samvit_mlp (HIP head forward +
    backward, sam_head_train.hip; head="torch" runs
    the head as torch ops instead, for comparison)."""
    net = renderer.net
    rows, image, depth, wsum = _FusedSamRows.apply(net.s_grid.embeddings, renderer, rays_o,
                                                    rays_d, cam_near_far, bg_color, view_width)
    head = head or "hip"
    if head == "torch":
        samvit = net.samvit_mlp(rows[:, :163])
    else:
        samvit = _SamHeadTrain.apply(rows, renderer, *_head_params(net))
    return {"samvit": samvit, "image": image, "depth": depth, "weights_sum": wsum}


# ----------------------------------------------------------- mask training --
class _FusedMaskTrain(torch.autograd.Function):
    """instance_mask_logits of a fused mask head in the --with_mask training
    step (nerf/utils.py:941-977 -> renderer.py:392-395, :451-452), forward and
    backward on the HIP kernels (mask_head_train.hip): for a 'default' head
    (exact fp32 MFMA) differentiable w.r.t. m_grid.embeddings and the three
    mask_mlp weights, for an 'adaptive' head (density, or rgb with
    sum_after_mlp) w.r.t. its six / eight mask_mlp weights -- the tensors the
    reference's loss reaches (weights, geo_feat and the grid_mlp / view_mlp
    intermediates are detached there).  image / depth / weights_sum come back
    without gradient.  params = (m_grid.embeddings, W0, W1, W2) for a 'default'
    head, the mask_mlp weights in order for an adaptive one."""

    @staticmethod
    def forward(ctx, renderer, rays_o, rays_d, cnf, bg, *params):
        N = rays_o.shape[0]
        dev = rays_o.device
        out = renderer.render(rays_o, rays_d, cnf, bg, keep_workspace=True, feats=False,
                              own_workspace=True, mask=True, mask_logits=False)
        ws, need, m, vw = out.pop("_workspace")
        m.with_mask = 2
        tneed = lib().samnerf_mask_train_workspace_size_model(ctypes.byref(m), N)
        tws = torch.empty(max(tneed, 1), dtype=torch.uint8, device=dev)
        logits = torch.empty(N, int(m.mask_out), device=dev)
        m.with_mask, m.view_width = 2, vw
        check(lib().samnerf_mask_train_forward(ctypes.byref(m), N, _ptr(logits), _ptr(ws), need, _ptr(tws),
                                               tneed, _stream(rays_o)), "mask_train_forward")
        ctx.state = (m, vw, ws, need, tws, tneed, list(renderer._keep))
        ctx.shapes = tuple(p.shape for p in params)
        ctx.kind = int(m.mask_kind)
        ctx.mark_non_differentiable(out["image"], out["depth"], out["weights_sum"])
        return logits, out["image"], out["depth"], out["weights_sum"]

    @staticmethod
    def backward(ctx, g_logits, g_img, g_depth, g_wsum):
        m, vw, ws, need, tws, tneed, _ = ctx.state
        g = g_logits.contiguous().float()          # bound: alive through the C call
        dev = g.device
        adaptive = ctx.kind != 0
        g_emb = None if adaptive else torch.zeros(ctx.shapes[0], device=dev)
        gw = [torch.empty(sh, device=dev) for sh in (ctx.shapes if adaptive else ctx.shapes[1:])]
        arr = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in gw])
        m.with_mask, m.view_width = 2, vw
        check(lib().samnerf_mask_train_backward(ctypes.byref(m), g.shape[0], _ptr(g), arr, _ptr(g_emb),
                                                _ptr(ws), need, _ptr(tws), tneed, _stream(g)),
              "mask_train_backward")
        return (None,) * 5 + ((*gw,) if adaptive else (g_emb, *gw))


def render_mask_train(renderer, rays_o, rays_d, cam_near_far=None, bg_color=None):
    """NeRFRenderer.run in train mode under grad with return_mask=1 for a fused
    mask head (the mask training step's render, utils.py:946-948): image,
    depth, weights_sum (no gradient) and instance_mask_logits with gradient to
    the head's trained tensors (_FusedMaskTrain): m_grid and mask_mlp for a
    'default' head, the mask_mlp Linears for an adaptive one."""
    net = renderer.net
    rays_o = rays_o.contiguous().float()
    rays_d = rays_d.contiguous().float()
    bg = 1.0 if bg_color is None else float(bg_color)
    cnf = None if cam_near_far is None else cam_near_far.contiguous().float()
    if mask_kind(net) == 0:
        skip = net.mask_mlp[0]
        params = (net.m_grid.embeddings, skip.net[0].weight, skip.net[1].weight, skip.net[2].weight)
    else:
        params = tuple(layer.weight for layer in net.mask_mlp)
    logits, image, depth, wsum = _FusedMaskTrain.apply(renderer, rays_o, rays_d, cnf, bg, *params)
    return {"image": image, "depth": depth, "weights_sum": wsum, "instance_mask_logits": logits}


# ------------------------------------------------------------ RGB training --
def rgb_train_params(net, with_prop):
    """The tensors the RGB training backward writes, in samnerf_rgb_grads order
    (NeRFNetwork.get_params groups, network.py:201-206); the proposal networks'
    only on the steps they train (renderer.py:290, utils.py:912-913)."""
    ps = [net.grid.embeddings] + [net.grid_mlp.net[i].weight for i in range(3)] + \
        [net.view_mlp.net[i].weight for i in range(3)]
    if with_prop:
        ps += [net.prop_encoders[0].embeddings, net.prop_encoders[1].embeddings] + \
            [net.prop_mlp[p].net[i].weight for p in range(2) for i in range(2)]
    return ps


class _FusedRGBTrain(torch.autograd.Function):
    """NeRFRenderer.run in train mode under grad for an RGB model
    (renderer.py:221-362) as samnerf_rgb_train_forward / _backward: outputs
    image, depth, weights_sum and the render's own losses (proposal_loss,
    distort_loss), differentiable w.r.t. every trained tensor; the Trainer's
    criterion and the entropy term stay torch ops on them."""

    @staticmethod
    def forward(ctx, renderer, rays_o, rays_d, cnf, bg, pert, with_prop, *params):
        N = rays_o.shape[0]
        dev = rays_o.device
        m = renderer.model()
        m.view_width = 0
        m.with_mask = 0
        need = lib().samnerf_rgb_train_workspace_size(ctypes.byref(m), N)
        ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        image = torch.empty(N, 3, device=dev)
        depth = torch.empty(N, device=dev)
        wsum = torch.empty(N, device=dev)
        weights = torch.empty(N, int(m.num_steps[2]), device=dev)
        losses = torch.zeros(2, device=dev)
        n_cnf = 0 if cnf is None else cnf.shape[0]
        try:
            for i in range(3):
                m.perturb[i] = None if pert is None else _param(pert[i], f"perturb[{i}]")
            check(lib().samnerf_rgb_train_forward(
                ctypes.byref(m), _ptr(rays_o), _ptr(rays_d), N, _ptr(cnf), n_cnf, float(bg), int(with_prop),
                _ptr(image), _ptr(depth), _ptr(wsum), _ptr(weights), _ptr(losses), _ptr(ws), need,
                _stream(rays_o)),
                "rgb_train_forward")
        finally:
            for i in range(3):
                m.perturb[i] = None
        ctx.state = (renderer, m, rays_o, rays_d, bg, pert, with_prop, ws, need, list(renderer._keep))
        ctx.shapes = [p.shape for p in params]
        # outputs the loss does not use arrive as None (no zero tensors to
        # read): only results['weights'] usually is
        ctx.set_materialize_grads(False)
        return image, depth, wsum, losses[0], losses[1], weights

    @staticmethod
    def backward(ctx, g_img, g_depth, g_wsum, g_prop, g_dist, g_weights):
        renderer, m, rays_o, rays_d, bg, pert, with_prop, ws, need, _ = ctx.state
        dev = rays_o.device
        N = rays_o.shape[0]
        # a loss without proposal_loss leaves the proposal networks' .grad None,
        # as autograd does (the final weights use detached bins)
        with_prop = with_prop and g_prop is not None
        # every converted gradient is bound to a local so that it stays alive
        # until the C call returns (a temporary's block could otherwise be
        # handed to the next conversion by the caching allocator)
        def conv(t):
            return None if t is None else t.contiguous().float()
        g_img = conv(g_img) if g_img is not None else torch.zeros(N, 3, device=dev)
        g_ws, g_dp, g_w = conv(g_wsum), conv(g_depth), conv(g_weights)   # None: no gradient (NULL)
        zero = torch.zeros((), device=dev)
        g_loss = torch.stack([(zero if g_prop is None else g_prop).reshape(()),
                              (zero if g_dist is None else g_dist).reshape(())]).float().contiguous()
        grads = [torch.empty(sh, device=dev) for sh in ctx.shapes]
        g = SamnerfRgbGrads()
        g.grid = grads[0].data_ptr()
        for i in range(3):
            g.grid_mlp[i] = grads[1 + i].data_ptr()
            g.view_mlp[i] = grads[4 + i].data_ptr()
        if with_prop:
            g.prop[0], g.prop[1] = grads[7].data_ptr(), grads[8].data_ptr()
            for q in range(2):
                for i in range(2):
                    g.prop_mlp[q][i] = grads[9 + 2 * q + i].data_ptr()
        try:
            for i in range(3):
                m.perturb[i] = None if pert is None else _param(pert[i], f"perturb[{i}]")
            check(lib().samnerf_rgb_train_backward(
                ctypes.byref(m), _ptr(rays_o), _ptr(rays_d), N, float(bg), int(with_prop), _ptr(g_img),
                _ptr(g_ws), _ptr(g_dp), _ptr(g_w), _ptr(g_loss),
                ctypes.byref(g), _ptr(ws), need, _stream(g_img)), "rgb_train_backward")
        finally:
            for i in range(3):
                m.perturb[i] = None
        if not with_prop:
            grads = grads[:7] + [None] * (len(grads) - 7)
        return (None,) * 7 + tuple(grads)


def render_rgb_train(renderer, rays_o, rays_d, cam_near_far=None, bg_color=None, perturb=False,
                     update_proposal=True):
    """The results dict of NeRFRenderer.run for an RGB model in train mode with
    grad (renderer.py:221-362): image, depth, weights_sum, num_points and --
    when lambda_proposal > 0 and update_proposal -- proposal_loss, when
    lambda_distort > 0 distort_loss, all differentiable on the HIP training
    kernels (rgb_train.hip)."""
    net = renderer.net
    opt = net.opt
    rays_o = rays_o.contiguous().float()
    rays_d = rays_d.contiguous().float()
    N = rays_o.shape[0]
    bg = 1.0 if bg_color is None else (float(bg_color) if not torch.is_tensor(bg_color) else
                                        float(bg_color.reshape(())))
    m = renderer.model()
    pert = None
    if isinstance(perturb, (tuple, list)) or perturb:
        pert = tuple(perturb) if isinstance(perturb, (tuple, list)) else \
            perturbed_positions(N, list(m.num_steps), rays_o.device)
        pert = tuple(t.contiguous().float() for t in pert)
    cnf = None if cam_near_far is None else cam_near_far.contiguous().float()
    with_prop = bool(update_proposal) and getattr(opt, "lambda_proposal", 0) > 0
    image, depth, wsum, prop_loss, dist_loss, weights = _FusedRGBTrain.apply(
        renderer, rays_o, rays_d, cnf, bg, pert, with_prop, *rgb_train_params(net, with_prop))
    out = {"num_points": N * int(m.num_steps[2]), "weights": weights, "weights_sum": wsum, "depth": depth,
           "image": image}
    if with_prop:
        out["proposal_loss"] = prop_loss
    if getattr(opt, "lambda_distort", 0) > 0:
        out["distort_loss"] = dist_loss
    return out
