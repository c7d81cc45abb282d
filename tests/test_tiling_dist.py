"""Multi-process band tiling (the N>1 path of bench.py) on CPU with the gloo backend, world_size 2 and 3."""
import os
import socket

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("height,world", [(1080, 1), (1080, 2), (1080, 8), (1080, 7), (64, 3), (5, 8), (1, 2)])
def test_bands_cover_rows_once(height, world):
    from synerfgine_amd.tiling import band_rows, tile_height
    seen = np.zeros(height, np.int32)
    th = tile_height(height, world)
    for r in range(world):
        r0, r1 = band_rows(height, r, world)
        assert 0 <= r0 <= r1 <= height and r1 - r0 <= th
        seen[r0:r1] += 1
    assert (seen == 1).all()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from synerfgine_amd.tiling import band_rows, gather_bands, tile_height
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = np.load(os.path.join(HERE, "golden", "frame_nerf_64.npz"))["rgba"]   # oracle-rendered 64x64 frame
        H, W, C = full.shape
        r0, r1 = band_rows(H, rank, world)
        th = tile_height(H, world)
        tile = torch.zeros((th, W, C), dtype=torch.float32)
        tile[: r1 - r0] = torch.from_numpy(full[r0:r1])        # this rank's band, as sng_render_frame(rows) leaves it
        frame = torch.empty((world * th, W, C), dtype=torch.float32)
        gather_bands(tile, frame)
        ok = bool(np.array_equal(frame[:H].numpy(), full))
        t = torch.tensor([1.0 if ok else 0.0])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)                # same reduction bench.py uses for timing
        q.put((rank, ok, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_band_gather_reassembles_frame(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok and agree == 1.0 for _, ok, agree in res)


def test_balance_bounds_equalises_cost():
    from synerfgine_amd.tiling import balance_bounds, even_bounds
    H, N = 1080, 8
    cost = np.ones(H)
    cost[300:700] = 60.0          # an object in the middle rows
    b = even_bounds(H, N)
    for _ in range(12):
        t = [cost[b[r]:b[r + 1]].sum() for r in range(N)]
        b = balance_bounds(H, b, t)
    t = [cost[b[r]:b[r + 1]].sum() for r in range(N)]
    assert b[0] == 0 and b[-1] == H and all(b[k] < b[k + 1] for k in range(N))
    assert max(t) / (sum(t) / N) < 1.15
    # equal cost stays (nearly) equal-height
    b2 = balance_bounds(H, even_bounds(H, N), [1.0] * N)
    assert max(abs(x - y) for x, y in zip(b2, even_bounds(H, N))) <= 1


def _root_worker(rank, world, port, bounds, q):
    import torch
    import torch.distributed as dist
    from synerfgine_amd.tiling import gather_to_root
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # the oracle-rendered 64x64 frame as RGBA8 words (the sng_final_rgba8 / sng_gather_rgba8 payload)
        full = np.load(os.path.join(HERE, "golden", "frame_nerf_64.npz"))["rgba"]
        words = np.ascontiguousarray((np.clip(full, 0, 1) * 255 + 0.5).astype(np.uint8)).view(np.int32)[..., 0]
        H, W = words.shape
        band = max(bounds[k + 1] - bounds[k] for k in range(world))
        r0, r1 = bounds[rank], bounds[rank + 1]
        tile = torch.full((band, W), -1, dtype=torch.int32)           # padding rows must not reach the frame
        tile[: r1 - r0] = torch.from_numpy(words[r0:r1])
        frame = torch.zeros((H, W), dtype=torch.int32) if rank == 0 else None
        out = gather_to_root(tile, bounds, frame)
        q.put((rank, out is None if rank else bool(np.array_equal(out.numpy(), words))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bounds", [[0, 9, 64], [0, 40, 41, 64], [0, 0, 64]], ids=["uneven2", "uneven3", "empty_band"])
def test_gloo_gather_to_root_reassembles_uneven_bands(bounds):
    """bench.py --gpus N --dist-backend gloo: the cost-balanced (uneven) bands reach rank 0's frame rows by their
    bounds, as sng_gather_rgba8 does over RCCL (comm.cpp); other ranks receive nothing."""
    import torch.multiprocessing as mp
    world = len(bounds) - 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_root_worker, args=(r, world, port, bounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok in res), res
