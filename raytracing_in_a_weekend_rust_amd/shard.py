"""Multi-GPU work split: frames per rank, or one frame's rows.

Weak scaling (bench.py default): an N-rank job renders N frames of the workload,
one whole frame per rank (frame_seed); no data-path collective.

Row-cyclic sharding of one frame (bench.py --scaling strong, BASELINE configs[3]):

Pixels are independent and each pixel's RNG stream depends only on its global
index (copy_reset chain, camera.rs:269-272), so any row partition reproduces the
single-GPU image bit-for-bit. Rows go to ranks cyclically (row r -> rank r % N)
because sky rows are ~3x cheaper than ground rows. The one exchange is a gather
of the row tiles (RCCL all_gather over xGMI on GPUs, gloo in CPU tests),
followed by an un-permute on the receiving rank.
"""
from __future__ import annotations


def frame_seed(seed: int, frame: int) -> int:
    """Render seed of frame `frame` of a multi-frame job. The reference seeds every
    render from the wall clock in ms (random.rs:16-22, camera.rs:255), so renders
    made one after another see consecutive seeds; frame 0 is the single-GPU
    workload itself."""
    return (seed + frame) % (1 << 128)


def rows_of(rank: int, world: int, height: int):
    """(row_begin, row_step, n_rows) of `rank`'s shard: rows rank, rank+world, ..."""
    return rank, world, len(range(rank, height, world))


def rows_max(world: int, height: int) -> int:
    return len(range(0, height, world))


def unpermute_index(world: int, height: int, device=None):
    """(src, dst) row indices: gathered[src[i]] is image row dst[i], where the
    gathered buffer holds each rank's tile padded to rows_max rows."""
    import torch

    rm = rows_max(world, height)
    src, dst = [], []
    for r in range(world):
        for k in range(len(range(r, height, world))):
            src.append(r * rm + k)
            dst.append(r + k * world)
    return (torch.tensor(src, dtype=torch.long, device=device),
            torch.tensor(dst, dtype=torch.long, device=device))


def gather_image(tile, world: int, height: int, gathered=None, image=None, index=None):
    """All-gather the padded (rows_max, W, 3) tiles of every rank and assemble
    the (height, W, 3) image. Collective: every rank must call it."""
    import torch
    import torch.distributed as dist

    rm = rows_max(world, height)
    assert tile.shape[0] == rm, "tile must be padded to rows_max rows"
    if gathered is None:
        gathered = torch.empty((world * rm,) + tuple(tile.shape[1:]), dtype=tile.dtype,
                               device=tile.device)
    dist.all_gather_into_tensor(gathered, tile)
    if index is None:
        index = unpermute_index(world, height, tile.device)
    src, dst = index
    if image is None:
        image = torch.empty((height,) + tuple(tile.shape[1:]), dtype=tile.dtype, device=tile.device)
    image.index_copy_(0, dst, gathered.index_select(0, src))
    return image
