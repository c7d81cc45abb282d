"""Multi-GPU frame tiling: one process per GPU renders a horizontal band, RCCL gathers the bands.

SURVEY.md §8e: rays are independent, so the frame shards into contiguous row bands with no
data-path collective; halo rows needed by normals (+-2) and NeRF shadows (+-r) are recomputed
inside sng_render_frame (capi.cpp render_frame), not exchanged.  The only exchange is the final
gather of the RGBA bands to every rank (all_gather_into_tensor over RCCL/xGMI; one ~1-8 MB tile
per peer at 1080p).
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
