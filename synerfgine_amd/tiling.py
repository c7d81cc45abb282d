"""Multi-GPU frame tiling: one process per GPU renders a horizontal band, RCCL gathers the bands.

SURVEY.md §8e: rays are independent, so the frame shards into contiguous row bands with no
data-path collective; halo rows needed by normals (+-2) and NeRF shadows (+-r) are recomputed
inside sng_render_frame (host_render.cpp render_frame), not exchanged.  The exchanges are the frame-wide
step schedule (comm.cpp) and the final gather of the RGBA8 bands to rank 0 (sng_gather_rgba8: grouped
ncclSend / ncclRecv over xGMI, ~1 MB per peer at 1080p); gather_to_root is its gloo rehearsal.
"""
import math


def band_rows(height, rank, world):
    """Rows [r0, r1) of `rank`'s band; all bands but the last have ceil(height / world) rows."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    tile = math.ceil(height / world)
    r0 = min(height, rank * tile)
    r1 = min(height, r0 + tile)
    return r0, r1


def tile_height(height, world):
    return math.ceil(height / world)


def gather_bands(tile, frame, group=None):
    """Gather equally sized band tiles [tile_h, W, C] of all ranks into frame [world*tile_h, W, C]."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":   # gloo has no all_gather_into_tensor
        world = dist.get_world_size(group)
        parts = list(frame.chunk(world, dim=0))
        dist.all_gather(parts, tile, group=group)
        return frame
    dist.all_gather_into_tensor(frame, tile, group=group)
    return frame


def assemble_bands(parts, bounds, frame):
    """Frame rows from the ranks' band tiles: part r holds its rows [bounds[r], bounds[r+1]) at the top of a tile
    padded to the tallest band (what sng_final_rgba8 of a band leaves in the tile)."""
    for r, part in enumerate(parts):
        frame[bounds[r]:bounds[r + 1]] = part[: bounds[r + 1] - bounds[r]]
    return frame


def gather_to_root(tile, bounds, frame=None, group=None):
    """The gloo (CPU) rehearsal of sng_gather_rgba8: every rank's band rows, the top rows of its padded `tile`, go
    to rank 0 only and land in rows [bounds[r], bounds[r+1]) of `frame` (rank 0: [height, ...]; other ranks may
    pass None).  Returns the frame on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    parts = [torch.empty_like(tile) for _ in range(world)] if rank == 0 else None
    dist.gather(tile, parts, dst=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return assemble_bands(parts, bounds, frame) if rank == 0 else None


def even_bounds(height, world):
    """Row boundaries [b0=0, b1, ..., b_world=height] of the equal-height bands."""
    return [band_rows(height, r, world)[0] for r in range(world)] + [height]


def balance_bounds(height, bounds, times, min_rows=8, damping=0.75):
    """Re-split rows so every band costs the same, from the previous split's per-band times.

    SURVEY.md §8e: sky rows are nearly free while rows through the NeRF object and the mesh cost
    ~100x more, so equal-height bands scale poorly.  The cost is modelled as piecewise constant per
    band (time / rows) and the cumulative cost is cut into equal parts; `damping` blends the new
    boundaries with the old ones so the iteration converges without oscillating.  Deterministic:
    every rank computes the same bounds from the same gathered times.
    """
    world = len(times)
    if world == 1:
        return [0, height]
    dens = []
    for r in range(world):
        rows = max(1, bounds[r + 1] - bounds[r])
        dens.append(max(float(times[r]), 1e-6) / rows)
    cum = [0.0]
    for r in range(world):
        cum.append(cum[-1] + dens[r] * (bounds[r + 1] - bounds[r]))
    total = cum[-1]
    new = [0]
    for k in range(1, world):
        target = total * k / world
        r = 0
        while r < world - 1 and cum[r + 1] < target:
            r += 1
        row = bounds[r] + (target - cum[r]) / dens[r]
        row = damping * row + (1.0 - damping) * bounds[k]
        new.append(int(round(row)))
    new.append(height)
    # monotone with at least min_rows per band (when the frame allows it)
    m = min(min_rows, height // world)
    for k in range(1, world):
        new[k] = max(new[k], new[k - 1] + m)
    for k in range(world - 1, 0, -1):
        new[k] = min(new[k], new[k + 1] - m)
    return new
