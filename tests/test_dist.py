"""Multi-process ray sharding + all-gather, world_size 2 on gloo (CPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _fake_render(o, d):
    # a per-ray function stands in for the renderer (no GPU here); exact
    # copies of the inputs so row placement is checked bit for bit
    return {"image": o.clone(), "depth": d[:, 0].clone(), "weights_sum": o[:, 1].clone(),
            "samvit": torch.cat([o, d], -1).repeat(1, 43)[:, :256]}


def _fake_render_tile(o, d, out_tile=None):
    # the out_tile form (FusedRenderer.render(out_tile=...), the layout of
    # samnerf_render_forward_tile): outputs written into the caller's rows
    r = _fake_render(o, d)
    if out_tile is None:
        return r
    out_tile[:, 0:3] = r["image"]
    out_tile[:, 3] = r["depth"]
    out_tile[:, 4] = r["weights_sum"]
    out_tile[:, 5:261] = r["samvit"]
    return {"image": out_tile[:, 0:3], "depth": out_tile[:, 3], "weights_sum": out_tile[:, 4],
            "samvit": out_tile[:, 5:261]}


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "segment-anything-nerf_amd"))
        from samnerf_amd.dist import render_sharded, render_view_sharded
        g = torch.Generator().manual_seed(0)
        o = torch.randn(n, 3, generator=g)
        d = torch.randn(n, 3, generator=g)
        out = render_sharded(_fake_render, o, d)
        ref = _fake_render(o, d)
        ok = all(torch.equal(out[k], ref[k]) for k in ref)
        # the pipelined per-view path: rows x W rays, chunked async all-gather
        H, W = 16, n // 16
        calls = []

        def ray_fn(row0, rows):
            calls.append((row0, rows))
            return o[row0 * W:(row0 + rows) * W], d[row0 * W:(row0 + rows) * W]

        view = render_view_sharded(_fake_render, ray_fn, H, W, chunks=4)
        ok = ok and all(torch.equal(view[k], ref[k][:H * W]) for k in ref)
        ok = ok and len(calls) == 4 and all(r == 2 for _, r in calls)
        # the cross-view pipeline: 3 views (shifted inputs), one gather in flight
        from samnerf_amd.dist import ShardedViewPipeline
        pipe = ShardedViewPipeline(_fake_render, H, W)
        got = []
        for v in range(3):
            def ray_fn_v(row0, rows, v=v):
                return (o[row0 * W:(row0 + rows) * W] + v, d[row0 * W:(row0 + rows) * W])
            pipe.submit(ray_fn_v)
            r_ = pipe.collect_ready()
            if r_ is not None:
                got.append(r_)
        got += pipe.flush()
        ok = ok and len(got) == 3
        for v, g in enumerate(got):
            refv = _fake_render(o[:H * W] + v, d[:H * W])
            ok = ok and all(torch.equal(g[k], refv[k]) for k in refv)
        # the same pipeline rendering into its slice of the gather buffer
        # (tile_cols): the band is never packed, the gather fills the buffer in place
        pipe = ShardedViewPipeline(_fake_render_tile, H, W, tile_cols=261)
        for v in range(3):
            def ray_fn_t(row0, rows, v=v):
                return (o[row0 * W:(row0 + rows) * W] - v, d[row0 * W:(row0 + rows) * W])
            pipe.submit(ray_fn_t)
        got = pipe.flush()
        ok = ok and len(got) == 3
        for v, g in enumerate(got):
            refv = _fake_render(o[:H * W] - v, d[:H * W])
            ok = ok and all(torch.equal(g[k], refv[k]) for k in refv)
        q.put((rank, ok, {k: tuple(v.shape) for k, v in out.items()}))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n", [4096, 1001])
def test_render_sharded_gloo_world2(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, shapes in res:
        assert ok, f"rank {rank} gathered wrong rows"
        assert shapes["image"] == (n, 3) and shapes["samvit"] == (n, 256)


def test_tile_cols_only_for_whole_tile_layouts():
    """samnerf_render_forward_tile always writes columns 0-4, so only
    the 3- and 4-key prefixes of (image, depth, weights_sum, samvit) describe a
    tile it fills; a 2-key prefix is refused at construction, not at the
    first submit."""
    import pytest
    from samnerf_amd.dist import ShardedViewPipeline
    with pytest.raises(ValueError, match="tile_cols"):
        ShardedViewPipeline(None, 8, 8, keys=("image", "depth"), tile_cols=4)
    with pytest.raises(ValueError, match="tile_cols"):
        ShardedViewPipeline(None, 8, 8, keys=("image", "depth", "weights_sum", "samvit"), tile_cols=260)
