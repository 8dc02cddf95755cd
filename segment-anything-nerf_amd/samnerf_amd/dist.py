"""Ray-sharded multi-GPU rendering: one process per GPU, RCCL all-gather.

Every ray does identical work (fixed 128/64/32 samples), so a
view is split into contiguous row bands of equal size -- perfectly balanced
with no data-path communication -- and the only exchange is one all-gather of
the packed per-ray output tile [rays_per_rank, 3 + 1 + 1 (+ 256)] fp32 so every
rank ends with the whole image/feature map.  With the `nccl`
backend (RCCL on ROCm) this is ncclAllGather over xGMI; `gloo` is used by the
CPU tests.
"""
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """Contiguous [start, stop) of n items for `rank` (first n % world ranks get
    one extra item)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def pack_outputs(out, keys):
    cols = []
    for k in keys:
        v = out[k]
        cols.append(v.reshape(v.shape[0], -1).float())
    return torch.cat(cols, dim=1)


def unpack_outputs(tile, keys, widths):
    res, c = {}, 0
    for k, w in zip(keys, widths):
        v = tile[:, c:c + w]
        res[k] = v.squeeze(1) if w == 1 else v
        c += w
    return res


def all_gather_rows(local, n_total, group=None):
    """Gather per-rank row blocks (possibly ragged by one row) into [n_total, C]."""
    world = dist.get_world_size(group)
    C = local.shape[1]
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    cap = max(b - a for a, b in sizes)
    padded = local.new_zeros(cap, C)
    padded[:local.shape[0]] = local
    if dist.get_backend(group) == "nccl":
        buf = local.new_empty(world * cap, C)
        dist.all_gather_into_tensor(buf, padded, group=group)
        parts = buf.view(world, cap, C)
    else:
        parts = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(parts, padded, group=group)
    return torch.cat([parts[r][:b - a] for r, (a, b) in enumerate(sizes)], dim=0)


def render_sharded(render_fn, rays_o, rays_d, keys=("image", "depth", "weights_sum", "samvit"),
                   group=None, gather=True):
    """Render this rank's band of rays with `render_fn(rays_o, rays_d) -> dict`
    and (optionally) all-gather the packed outputs.  rays_* are the full [N,3]
    view on every rank (or only the local band if `gather` knows N)."""
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
