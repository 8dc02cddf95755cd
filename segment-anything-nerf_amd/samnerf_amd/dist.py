"""Ray-sharded multi-GPU rendering: one process per GPU, RCCL all-gather.

Every ray does identical work (fixed 128/64/32 samples), so a
view is split into contiguous row bands of equal size -- perfectly balanced
with no data-path communication -- and the only exchange is the all-gather
of the packed per-ray outputs [rays, 3 + 1 + 1 (+ 256)] fp32 so every rank
ends with the whole image / feature map.  With the `nccl`
backend (RCCL on ROCm) this is ncclAllGather over xGMI; `gloo` is used by the
CPU tests.

`render_view_sharded` pipelines the band in chunks: the all-gather of chunk
i is issued asynchronously (RCCL runs on its own stream after the chunk's
kernels) while chunk i+1 renders, so communication hides behind compute.
"""
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """Contiguous [start, stop) of n items for `rank` (first n % world ranks get
    one extra item)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


KEYS_ALL = ("image", "depth", "weights_sum", "samvit")
KEY_WIDTHS = (3, 1, 1, 256)


def pack_outputs(out, keys):
    return torch.cat([out[k].reshape(out[k].shape[0], -1).float() for k in keys], dim=1)


def unpack_outputs(tile, keys, widths):
    res, c = {}, 0
    for k, w in zip(keys, widths):
        v = tile[:, c:c + w]
        res[k] = v.squeeze(1) if w == 1 else v
        c += w
    return res


class _Done:
    """Work handle of a collective that has already completed."""

    def wait(self):
        return True


def _all_gather(buf_out, local, group, async_op=False):
    """all_gather of equal-size row blocks into buf_out [world * n, C].  With
    RCCL (`nccl`) this is one all_gather_into_tensor over xGMI.  Under `gloo`
    (CPU tests, and the single-GPU rehearsal of the multi-rank bench) device
    tensors are staged through host memory, synchronously."""
    if dist.get_backend(group) == "nccl":
        return dist.all_gather_into_tensor(buf_out, local, group=group, async_op=async_op)
    world = dist.get_world_size(group)
    if local.is_cuda:
        host = buf_out.new_empty(buf_out.shape, device="cpu")
        parts = list(host.chunk(world, 0))
        dist.all_gather(parts, local.cpu(), group=group)
        buf_out.copy_(host)
        return _Done() if async_op else None
    parts = list(buf_out.chunk(world, 0))
    return dist.all_gather(parts, local, group=group, async_op=async_op)


def all_gather_rows(local, n_total, group=None):
    """Gather per-rank row blocks (possibly ragged by one row) into [n_total, C]."""
    world = dist.get_world_size(group)
    C = local.shape[1]
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    cap = max(b - a for a, b in sizes)
    padded = local.new_zeros(cap, C)
    padded[:local.shape[0]] = local
    buf = local.new_empty(world * cap, C)
    _all_gather(buf, padded, group)
    parts = buf.view(world, cap, C)
    return torch.cat([parts[r][:b - a] for r, (a, b) in enumerate(sizes)], dim=0)


def render_sharded(render_fn, rays_o, rays_d, keys=("image", "depth", "weights_sum", "samvit"),
                   group=None, gather=True):
    """Render this rank's contiguous block of the given rays with
    `render_fn(rays_o, rays_d) -> dict` and (optionally) all-gather the packed
    outputs back into the original ray order."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    N = rays_o.shape[0]
    a, b = shard_range(N, rank, world)
    out = render_fn(rays_o[a:b], rays_d[a:b])
    keys = [k for k in keys if k in out]
    widths = [out[k].reshape(out[k].shape[0], -1).shape[1] for k in keys]
    if not gather:
        return out
    full = all_gather_rows(pack_outputs(out, keys), N, group)
    return unpack_outputs(full, keys, widths)


def render_view_sharded(render_fn, ray_fn, H, W, keys=("image", "depth", "weights_sum", "samvit"),
                        chunks=4, group=None):
    """Strong-scaled render of one HxW view over the ranks of `group`.

    ray_fn(row0, rows) -> (rays_o, rays_d) for pixel rows [row0, row0+rows);
    render_fn(rays_o, rays_d) -> dict of per-ray outputs.  Each rank takes the
    row band `shard_range(H, rank, world)` (H must split evenly so every
    all-gather has equal blocks), renders it in `chunks` row chunks and
    all-gathers each chunk asynchronously behind the next chunk's rendering.
    Returns the full view's outputs in image order on every rank."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if H % world:
        raise ValueError(f"H={H} must be divisible by the world size {world}")
    band = H // world
    chunks = max(1, min(chunks, band))
    while band % chunks:
        chunks -= 1
    crow = band // chunks
    r0 = rank * band
    pending, bufs = [], []
    widths = None
    for c in range(chunks):
        ro, rd = ray_fn(r0 + c * crow, crow)
        out = render_fn(ro, rd)
        ks = [k for k in keys if k in out]
        if widths is None:
            keys = ks
            widths = [out[k].reshape(out[k].shape[0], -1).shape[1] for k in keys]
        tile = pack_outputs(out, keys)
        buf = tile.new_empty(world * tile.shape[0], tile.shape[1])
        pending.append(_all_gather(buf, tile, group, async_op=True))
        bufs.append(buf)
    for p in pending:
        p.wait()
    n_c = crow * W
    C = bufs[0].shape[1]
    # bufs[c] = [world, n_c, C] (rank-major); image order is (rank, chunk, ray)
    full = torch.stack([b.view(world, n_c, C) for b in bufs], dim=1).reshape(world * chunks * n_c, C)
    return unpack_outputs(full, keys, widths)


class ShardedViewPipeline:
    """Strong-scaled rendering of a stream of views with the all-gather of
    view i running behind the rendering of view i+1.

        pipe = ShardedViewPipeline(render_fn, H, W)
        for view in views:
            pipe.submit(ray_fn_for(view))     # render this rank's band, start the gather
            done = pipe.collect_ready()       # outputs of the previous view, or None
        last = pipe.flush()

    submit() only enqueues GPU work (kernels on the current stream, the
    collective on RCCL's stream); collect_ready()/flush() make the current
    stream wait for the oldest gather and return its outputs in image order.
    One full-size launch per view and rank (no chunking): the communication
    hides behind the next view's kernels instead of shrinking them.

    codec = "fp32" gathers the outputs as they are (1,044 B per ray with the
    SAM features).  codec = "q16" gathers the transport records of
    ops.tile_encode (tile_codec.hip: 536 B per ray; image / depth /
    weights_sum exact, samvit as int16 with a per-ray power-of-two scale,
    |error| <= 2^-14 of the ray's max |samvit|); each rank's own band is put
    back in fp32 after decoding, so only the other ranks' copies carry the
    quantisation.  q16 needs CUDA outputs with samvit (there is no CPU codec)."""

    def __init__(self, render_fn, H, W, keys=("image", "depth", "weights_sum", "samvit"),
                 group=None, depth=1, codec="fp32", tile_cols=None):
        """tile_cols (fp32 transport): render_fn accepts out_tile= (as
        FusedRenderer.render) and writes a band's outputs as rows of this many
        columns (261 with samvit, 5 without; samnerf_render_forward_tile's
        layout = `keys` in order) -- straight into this rank's slice of the
        gather buffer, which the all-gather then fills in place: no pack copy
        of the band before the collective.  None: render into separate
        tensors and pack them (any render_fn)."""
        if codec not in ("fp32", "q16"):
            raise ValueError(f"codec must be 'fp32' or 'q16', got {codec!r}")
        # samnerf_render_forward_tile always writes columns 0-4 (and 5-260 when
        # the model has SAM features and feats=True): only the 3- and 4-key
        # prefixes describe a tile it fills; tile_cols = 5 needs a
        # render_fn with feats=False on a with_sam model
        if tile_cols is not None and (codec != "fp32" or len(keys) not in (3, 4)
                                      or tuple(keys) != KEYS_ALL[:len(keys)]
                                      or tile_cols != sum(KEY_WIDTHS[:len(keys)])):
            raise ValueError("tile_cols: fp32 transport of (image, depth, weights_sum[, samvit]) only")
        self.render_fn, self.H, self.W = render_fn, H, W
        self.keys, self.group, self.depth, self.codec = keys, group, depth, codec
        self.tile_cols = tile_cols
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if H % self.world:
            raise ValueError(f"H={H} must be divisible by the world size {self.world}")
        self.band = H // self.world
        self.inflight = []
        self.side = None

    def submit(self, ray_fn, render_fn=None):
        ro, rd = ray_fn(self.rank * self.band, self.band)
        if self.tile_cols is not None:
            n = ro.shape[0]
            buf = torch.empty(self.world * n, self.tile_cols, device=ro.device)
            own = buf[self.rank * n:(self.rank + 1) * n]
            out = (render_fn or self.render_fn)(ro, rd, out_tile=own)
            keys = list(self.keys)
            widths = list(KEY_WIDTHS[:len(keys)])
            work = _all_gather(buf, own, self.group, async_op=True)   # in place
            self.inflight.append((work, buf, own, keys, widths, out))
            return
        out = (render_fn or self.render_fn)(ro, rd)
        keys = [k for k in self.keys if k in out]
        widths = [out[k].reshape(out[k].shape[0], -1).shape[1] for k in keys]
        if self.codec == "q16":
            # encode + gather (+ later decode) on a side stream, ordered after
            # this view's kernels, so they overlap the next view's
            from .ops import tile_encode
            if keys != ["image", "depth", "weights_sum", "samvit"]:
                raise RuntimeError("q16 codec: needs image, depth, weights_sum and samvit outputs")
            dev = out["samvit"].device
            if self.side is None:
                self.side = torch.cuda.Stream(dev)
            self.side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self.side):
                tile = tile_encode(out)
                buf = tile.new_empty(self.world * tile.shape[0], tile.shape[1])
                work = _all_gather(buf, tile, self.group, async_op=True)
            for k in keys:
                out[k].record_stream(self.side)
        else:
            tile = pack_outputs(out, keys)
            buf = tile.new_empty(self.world * tile.shape[0], tile.shape[1])
            work = _all_gather(buf, tile, self.group, async_op=True)
        self.inflight.append((work, buf, tile, keys, widths, out))

    def _pop(self):
        work, buf, _tile, keys, widths, own = self.inflight.pop(0)
        if self.codec == "fp32":
            work.wait()
            return unpack_outputs(buf, keys, widths)      # rank-major bands = image order
        # Decode on the side stream, behind the collective; the caller's
        # stream waits for it only before the work it queues after this call.
        from .ops import tile_decode
        cur = torch.cuda.current_stream(buf.device)
        with torch.cuda.stream(self.side):
            work.wait()
            res = tile_decode(buf)
            n = own["depth"].shape[0]
            for k in keys:                                 # this rank's band stays exact
                res[k][self.rank * n:(self.rank + 1) * n] = own[k]
        cur.wait_stream(self.side)
        for v in res.values():
            v.record_stream(cur)
        return res

    def collect_ready(self):
        """Outputs of the oldest view once more than `depth` views are in flight."""
        return self._pop() if len(self.inflight) > self.depth else None

    def flush(self):
        outs = []
        while self.inflight:
            outs.append(self._pop())
        return outs
