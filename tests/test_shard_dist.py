"""Multi-rank paths on the CPU over gloo (world_size 2 and 3), with the oracle (the
GPU kernel's checker) as the renderer:
- strong (bench.py default): each rank renders its row-cyclic shard, the tiles are
  all-gathered and un-permuted by bench.py's own step code (shard.StepPlan /
  shard.step), and the result equals the unsharded image bit-for-bit;
- weak (bench.py --scaling weak): rank r renders frame r of the job at
  shard.frame_seed(SEED, r), frame 0 being the single-GPU workload."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raytracing_in_a_weekend_rust_amd import shard

H, W, S, SEED = 23, 31, 2, 4242


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from oracle import pyoracle as py
    from tests.golden.make_golden import c_camera, c_scene
    pc, objs = py.scene_builtin("complex", SEED, H, W, 20)
    sph, mat = c_scene(objs)
    return c_camera(pc), sph, mat, len(objs)


def _worker(rank, world, port, out):
    """One rank of bench.py's default N>1 step (shard.StepPlan + shard.step), with the
    oracle rendering the rank's rows in place of the GPU."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle_ctypes as orc
    cam, sph, mat, n = _scene()
    plan = shard.StepPlan(world, rank, H, W, False, SEED, torch.float64, "cpu")
    assert plan.describe() == f"row-cyclic x{world} + rccl all_gather"

    def render_tile(pl):
        rb, step, nr = pl.shard
        tile_np, _ = orc.render(cam, sph, n, mat, n, S, pl.render_seed, rows=(rb, step, nr), nthreads=2)
        pl.tile[:nr] = torch.from_numpy(tile_np)

    img = shard.step(plan, render_tile)
    if rank == 0:
        np.save(out, img.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_cyclic_gather_reassembles_image(world, tmp_path):
    from oracle import oracle_ctypes as orc
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    cam, sph, mat, n = _scene()
    full, _ = orc.render(cam, sph, n, mat, n, S, SEED, nthreads=2)
    assert np.array_equal(got, full)


def test_shard_rows_cover_image_once():
    for world in (1, 2, 4, 8):
        seen = []
        for r in range(world):
            b, step, n = shard.rows_of(r, world, 675)
            seen += list(range(b, b + n * step, step))
        assert sorted(seen) == list(range(675))
        src, dst = shard.unpermute_index(world, 675)
        assert sorted(dst.tolist()) == list(range(675))


def _frame_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle_ctypes as orc
    cam, sph, mat, n = _scene()
    plan = shard.StepPlan(world, rank, H, W, True, SEED, torch.float64, "cpu")
    assert plan.shard == (0, 1, H) and not plan.collective

    def render_tile(pl):
        fb, _ = orc.render(cam, sph, n, mat, n, S, pl.render_seed, nthreads=2)
        pl.tile[:] = torch.from_numpy(fb)

    frame = shard.step(plan, render_tile).clone()
    frames = [torch.zeros_like(frame) for _ in range(world)]
    dist.all_gather(frames, frame)  # the test's check only: the bench's weak path has no collective
    if rank == 0:
        np.save(out, torch.stack(frames).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_frame_per_rank_weak_scaling(tmp_path):
    from oracle import oracle_ctypes as orc
    world = 2
    out = str(tmp_path / "frames.npy")
    mp.spawn(_frame_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    cam, sph, mat, n = _scene()
    assert shard.frame_seed(SEED, 0) == SEED
    for f in range(world):
        ref, _ = orc.render(cam, sph, n, mat, n, S, shard.frame_seed(SEED, f), nthreads=2)
        assert np.array_equal(got[f], ref)
    assert not np.array_equal(got[0], got[1])  # independent frames, not replicas


def test_group_devices_for_plain_bench_command():
    """bench.py --gpus N without a launcher: the first N devices, or the visible ones
    repeated round-robin (labelled: not a scaling point)."""
    assert shard.group_devices(8, 8) == ([0, 1, 2, 3, 4, 5, 6, 7], False)
    assert shard.group_devices(2, 8) == ([0, 1], False)
    assert shard.group_devices(4, 1) == ([0, 0, 0, 0], True)
    assert shard.group_devices(3, 2) == ([0, 1, 0], True)
    with pytest.raises(ValueError):
        shard.group_devices(2, 0)


def test_group_rows_match_rank_rows():
    """An rtw_group entry i renders the rows rank i of a torchrun split renders
    (rows_of), into tiles padded to rows_max: the un-permute maps tile row k of
    entry i to image row i + k*N, covering every row once."""
    for world, h in [(1, 5), (2, 675), (3, 7), (8, 675), (5, 3)]:
        n = min(world, h)
        seen = []
        for i in range(n):
            b, step, rows = shard.rows_of(i, n, h)
            assert rows <= shard.rows_max(n, h)
            seen += [b + k * step for k in range(rows)]
        assert sorted(seen) == list(range(h))
