"""Multi-GPU work split: one frame's rows, or frames per rank.

Row-cyclic sharding of one frame (bench.py default, BASELINE configs[3]):

Pixels are independent and each pixel's RNG stream depends only on its global
index (copy_reset chain, camera.rs:269-272), so any row partition reproduces the
single-GPU image bit-for-bit. Rows go to ranks cyclically (row r -> rank r % N)
because sky rows are ~3x cheaper than ground rows. The one exchange is a gather
of the row tiles (RCCL all_gather over xGMI on GPUs, gloo in CPU tests),
followed by an un-permute on the receiving rank.

Weak scaling (bench.py --scaling weak): an N-rank job renders N frames of the
workload, one whole frame per rank (frame_seed); no data-path collective.

StepPlan + step() are what bench.py runs per timed step; tests/test_shard_dist.py
drives the same code over gloo with the oracle standing in for the GPU render.
"""
from __future__ import annotations


def group_devices(n: int, visible: int):
    """Device entries of a one-process N-GPU group (bench.py --gpus N without
    torchrun): the first N devices, or -- on a box with fewer GPUs -- the visible
    ones repeated round-robin (entries then share a GPU: a rehearsal of the N-way
    split and its gather, not a scaling point). Returns (devices, repeated)."""
    if n < 1 or visible < 1:
        raise ValueError(f"need n >= 1 and a visible device (n={n}, visible={visible})")
    devs = [i % visible for i in range(n)]
    return devs, n > visible


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


class StepPlan:
    """One rank's share of a bench step: its shard, render seed, device tile and --
    for N>1 strong scaling -- the gather buffers and the assembled image."""

    def __init__(self, world: int, rank: int, height: int, width: int, weak: bool, seed: int,
                 dtype, device, collective: bool = True):
        import torch

        self.world, self.rank, self.height, self.weak = world, rank, height, weak
        if weak:  # frame `rank` of an N-frame job, the whole image on this rank
            self.shard = (0, 1, height)
            rows = height
            self.render_seed = frame_seed(seed, rank)
        else:  # row-cyclic shard of the one frame
            self.shard = rows_of(rank, world, height)
            rows = rows_max(world, height)  # tiles padded to the same row count
            self.render_seed = seed
        self.tile = torch.zeros((rows, width, 3), dtype=dtype, device=device)
        self.collective = collective and world > 1 and not weak
        if self.collective:
            self.gathered = torch.empty((world * rows, width, 3), dtype=dtype, device=device)
            self.image = torch.empty((height, width, 3), dtype=dtype, device=device)
            self.index = unpermute_index(world, height, device)
        else:
            self.image = self.tile

    def gather(self):
        if self.collective:
            gather_image(self.tile, self.world, self.height, self.gathered, self.image, self.index)
        return self.image

    def describe(self) -> str:
        if self.weak:
            return f"frame-per-rank x{self.world} (render seed SEED+rank), no collective"
        return f"row-cyclic x{self.world}" + (" + rccl all_gather" if self.world > 1 else "")


def step(plan: StepPlan, render_tile, after_render=None):
    """One bench step: render this rank's rows into plan.tile, then the gather."""
    render_tile(plan)
    if after_render is not None:
        after_render()
    return plan.gather()
