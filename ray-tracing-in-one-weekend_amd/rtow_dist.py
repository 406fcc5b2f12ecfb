"""Multi-GPU frame assembly: interleaved row bands + one gather.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
MI355X; "gloo" on CPU for the tests).  Rank r renders the rows
    ((b * world) + r) * row_block + k,   b = 0, 1, ...,  k < row_block
into a contiguous local tile (local_rows x W x 3 fp32, equal on every rank;
rows past the image are padding), rank 0 gathers the tiles with a single
gather and de-interleaves them.  The RNG is keyed by the global pixel index,
so the assembled image is bit-identical for any world size.

Why interleaved bands: sky rows are cheap and ground rows expensive, so 8
contiguous bands give max/mean work 1.35 (speed-up capped at 5.9x on 8 GPUs)
while interleaving gives 1.02 (measured on the reference).
"""
import numpy as np

import rtow


def partition(width, height, spp, world, rank, row_block=8, **kw):
    """rt_params for `rank` of `world` (kw: max_depth, seed, flags)."""
    return rtow.make_params(width, height, spp, rank=rank, world=world, row_block=row_block, **kw)


def assemble(tiles, height, world, row_block=8):
    """tiles: [world, local_rows, W, 3] (rank order) -> frame [H, W, 3]."""
    tiles = np.asarray(tiles)
    w = tiles.shape[2]
    frame = np.zeros((height, w, 3), tiles.dtype)
    for r in range(world):
        p = rtow.make_params(w, height, 1, rank=r, world=world, row_block=row_block)
        rows = rtow.local_to_global_rows(p)
        keep = rows < height
        frame[rows[keep]] = tiles[r][keep]
    return frame


def gather_tiles(tile, world, rank, dst=0):
    """torch.distributed gather of equal-size tiles to `dst` (one collective).

    Returns the stacked [world, ...] tensor on dst, None elsewhere."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return tile.unsqueeze(0)
    out = [torch.empty_like(tile) for _ in range(world)] if rank == dst else None
    dist.gather(tile, out, dst=dst)
    return torch.stack(out) if rank == dst else None


def render_distributed(render_tile, width, height, spp, world, rank, row_block=8, **kw):
    """Render one frame across `world` ranks.

    render_tile(params) -> torch tensor [local_rows, W, 3] (device or CPU).
    Returns the assembled frame (numpy) on rank 0, None elsewhere."""
    p = partition(width, height, spp, world, rank, row_block, **kw)
    tile = render_tile(p)
    stacked = gather_tiles(tile, world, rank)
    if rank != 0:
        return None
    return assemble(stacked.cpu().numpy(), height, world, row_block)
