#!/usr/bin/env python3
"""Benchmark of the MI355X sampling path on BASELINE.json's headline workload.

Workload (BASELINE.json metric / configs[3]): the book's final random-spheres
scene (raytracing::complex, raytracing/mod.rs:54-126; 486 spheres at the fixed
scene seed), 1200x675, spp=500 -> samples_sqrt 23 (529 spp, the reference API
takes samples_sqrt), max_depth 50, f64 parity mode (bit-identical to the
reference restatement). One step = one whole-image render (Camera::threaded_render
equivalent) with the scene already resident in HBM.

N>1 (one rank per GPU): by default weak scaling -- the job renders N frames, rank r
frame r (render seed SEED + r, shard.frame_seed), each a full 1200x675 spp-529
image, with no data-path collective (frames are independent).
`--scaling strong` renders the ONE frame row-cyclically sharded over the ranks and
gathered over RCCL (all_gather of the row tiles) inside the timed step: BASELINE
configs[3]'s scaling curve, whose per-rank times the serial per-pixel RNG chains
bound.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line (contract in the task statement). The cpu_baseline
leg times the C oracle (test infrastructure, kind "port") on a bounded row
sample of the same workload on this host, at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch  # first: librtw then shares torch's HIP runtime (same soname)
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import raytracing_in_a_weekend_rust_amd as rtw  # noqa: E402
from raytracing_in_a_weekend_rust_amd import shard  # noqa: E402

SEED = rtw.DEFAULT_SEED
W, H, SQRT, DEPTH = 1200, 675, 23, 50
FLOP_PER_TEST = 17  # oc 3, half_b 5, c 6 (r*r hoisted), disc 3
FLOP_PER_VISIT = 20  # BVH walk step: slab test 6 FMA + 10 min/max, or the 17-FLOP sphere filter
FP32_VECTOR_PEAK = 157.3  # TFLOP/s, MI355X spec (MI355X_MICROARCH.md chip table)
FP64_VECTOR_PEAK = 78.6   # TFLOP/s, MI355X spec
PMC_FILE = os.path.join(HERE, "profiles", "pmc_traffic.json")
INSTS_FILE = os.path.join(HERE, "profiles", "pmc_insts.json")
GPU_CLOCK_HZ = 2.4e9  # MI355X peak engine clock (MI355X_MICROARCH.md)
# gfx950 VALU issue (MI355X_MICROARCH.md cycle constants): a wave64 f32/int VALU
# instruction occupies the 32-lane SIMD for 2 cycles; f64 FMA/MUL/ADD run at half
# rate (4 cycles: FP64 vector peak = 1/2 FP32); one wave alone issues at most one
# VALU instruction per 4 cycles.
VALU_CYCLES = 2
VALU_CYCLES_F64 = 4


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--samples-sqrt", type=int, default=SQRT)
    p.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                   help="N>1: weak = one whole frame per rank (seed SEED+rank), no collective; "
                        "strong = the one frame row-cyclically sharded + RCCL all_gather")
    p.add_argument("--mode", choices=("parity", "fast"), default="parity",
                   help="parity = f64 bit-exact (the headline); fast = the f32 mode with "
                        "independent per-sample streams (statistical parity, tests/test_gpu_fast.py)")
    p.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the CPU leg")
    p.add_argument("--e2e", type=int, default=1,
                   help="0 disables the end-to-end leg (one-shot ABI call with host buffers + PPM)")
    p.add_argument("--cpu-row-stride", type=int, default=0,
                   help="oracle renders every k-th row (0 = auto, ~10-30 s)")
    return p.parse_args()


def end_to_end(cam, sph, ns, mt, nm, s, seed, fast, kernel_ms):
    """SURVEY.md 8(d)'s end-to-end figure, outside the timed region: the one-shot
    rtw_threaded_render(_fast) (scene upload, seeds, render, framebuffer download to a
    host buffer: the reference's Camera::threaded_render, camera.rs:223-352) and then
    the PPM text (Color::wire_full_file, color.rs:196-247). One untimed call first
    (device context, allocations), then one timed call."""
    one_shot = rtw.render_flat_fast if fast else rtw.render_flat
    one_shot(cam, sph, ns, mt, nm, s, seed)
    t0 = time.perf_counter()
    fb, _ = one_shot(cam, sph, ns, mt, nm, s, seed)
    t1 = time.perf_counter()
    ppm = rtw.format_ppm(fb)
    t2 = time.perf_counter()
    render_ms, ppm_ms = (t1 - t0) * 1e3, (t2 - t1) * 1e3
    samples = W * H * (s * s if s else 1)
    return {"render_ms": round(render_ms, 3), "ppm_ms": round(ppm_ms, 3), "ppm_bytes": len(ppm),
            "host_overhead_ms": round(render_ms - kernel_ms, 3),
            "value": round(samples / ((render_ms + ppm_ms) / 1e3) / 1e6, 3), "unit": "Msamples/s",
            "note": "one-shot ABI call with host buffers (PCIe upload/download, seeds, render) + PPM "
                    "text; host_overhead_ms = render_ms - resident kernel_ms. Not `value`"}


def available_parallelism():
    """What the reference's pool would size itself to: Camera::threaded_render uses
    ThreadPoolBuilder::with_max_threads() (camera.rs:253) = Rust's
    std::thread::available_parallelism(), which on Linux is the CPU-affinity count
    capped by the cgroup CPU quota (cgroup v2 cpu.max, or v1 cfs_quota/period).
    Returns (threads, how it was derived)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(per))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    n = min(aff, quota) if quota else aff
    how = (f"available_parallelism(): min(affinity {aff}, cgroup CPU quota {quota})" if quota
           else f"available_parallelism(): affinity {aff} (no cgroup CPU quota)")
    return n, how


def cpu_baseline(cam, sph, ns, mt, nm, s, stride):
    """Oracle (C restatement) on a row sample, ref-faithful scheduler: one job per
    pixel pulled by `threads` workers, dyn dispatch + Arc-refcount traffic as in
    camera.rs:269-292 / sphere.rs:69."""
    from oracle import oracle_ctypes as orc  # test infrastructure: checker/baseline only

    # the reference's own pool size on this host (not a cap of ours)
    threads, how = available_parallelism()
    if os.environ.get("RTW_CPU_THREADS"):
        threads, how = int(os.environ["RTW_CPU_THREADS"]), "RTW_CPU_THREADS override"
    if stride <= 0:  # ~4 rows per thread: ~15 s of CPU work at ~0.16 Msamples/s/core
        stride = max(1, int(round(cam.img_height / (4 * threads))))
    n_rows = len(range(0, cam.img_height, stride))
    t0 = time.perf_counter()
    _, seg = orc.render(cam, sph, ns, mt, nm, s, SEED, rows=(0, stride, n_rows),
                        nthreads=threads, scheduler=0)
    dt = time.perf_counter() - t0
    samples = n_rows * cam.img_width * (s * s if s else 1)
    # also the "clean" scheduler (rows pulled by the workers, direct
    # calls, no per-pixel job/refcount overhead), on the same sampled rows
    c_stride = stride
    c_rows = len(range(0, cam.img_height, c_stride))
    t0 = time.perf_counter()
    orc.render(cam, sph, ns, mt, nm, s, SEED, rows=(0, c_stride, c_rows), nthreads=threads, scheduler=1)
    c_dt = time.perf_counter() - t0
    c_samples = c_rows * cam.img_width * (s * s if s else 1)
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"rows 0::{stride} ({n_rows} rows x {cam.img_width} px x {s * s} spp, "
                      f"{samples / 1e6:.1f} Msamples) of the same image, {dt:.1f} s, "
                      f"ref-faithful per-pixel jobs, {os.cpu_count()} host cpus visible",
            "threads_rule": how,
            "clean_scheduler": {"value": c_samples / c_dt / 1e6, "unit": "Msamples/s", "cores": threads,
                                "sample": f"rows 0::{c_stride} ({c_rows} rows), {c_dt:.1f} s, row jobs, "
                                          "direct calls"}}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N>1 needs torchrun --nproc-per-node N (one rank per GPU)")
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    s = a.samples_sqrt
    cam, sph, ns, mt, nm = rtw.builtin_scene("complex", SEED, H, W, DEPTH)
    n_off = s * s if s else 1
    weak = a.scaling == "weak"
    if weak:  # frame `rank` of an N-frame job, the whole image on this rank
        rb, rstep, rows_local, rm = 0, 1, H, H
        render_seed = shard.frame_seed(SEED, rank)
    else:  # row-cyclic shard of the one frame
        rb, rstep, rows_local = shard.rows_of(rank, world, H)
        rm = shard.rows_max(world, H)
        render_seed = SEED
    sess = rtw.Session(local)
    sess.set_scene(sph, ns, mt, nm)
    dev = torch.device("cuda", local)
    fast = a.mode == "fast"
    fdt = torch.float32 if fast else torch.float64
    fb = torch.zeros((rm, W, 3), dtype=fdt, device=dev)  # padded tile
    render = sess.render_fast if fast else sess.render
    if world > 1 and not weak:
        gathered = torch.empty((world * rm, W, 3), dtype=fdt, device=dev)
        image = torch.empty((H, W, 3), dtype=fdt, device=dev)
        index = shard.unpermute_index(world, H, dev)
    stream = torch.cuda.current_stream(dev)
    kernel_ms = []

    def step(record):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        render(cam.raw, s, render_seed, fb.data_ptr(), stream=stream.cuda_stream,
               shard=(rb, rstep, rows_local))
        ev1.record(stream)
        if world > 1 and not weak:  # RCCL all_gather of the row tiles + un-permute
            shard.gather_image(fb, world, H, gathered, image, index)
        if record:
            kernel_ms.append((ev0, ev1))

    for _ in range(a.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = sess.stats()  # last render: deterministic counters of this rank's shard
    kms = sum(e0.elapsed_time(e1) for e0, e1 in kernel_ms) / max(1, len(kernel_ms))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frames = world if weak else 1
    total_samples = frames * W * H * n_off * a.steps
    value = total_samples / elapsed / 1e6
    # `achieved` = SURVEY 8(d)'s algorithmic work: segments x N spheres x 17 FLOP (the
    # reference's f64 brute-force Scene::hit) per launch over the kernel time. The
    # exact BVH does not execute it: its executed work (walk visits ~20 FLOP each,
    # f32, + exact f64 sphere tests 17 each) is reported beside it
    brute_flop = st.sphere_tests * FLOP_PER_TEST
    if st.accel == 2:
        exec_flop = st.node_visits * FLOP_PER_VISIT + st.exact_tests * FLOP_PER_TEST
    else:
        exec_flop = brute_flop
    achieved = brute_flop / (kms / 1e3) / 1e12
    peak = FP32_VECTOR_PEAK if fast else FP64_VECTOR_PEAK
    executed = exec_flop / (kms / 1e3) / 1e12
    valu = None  # VALU issue utilisation from the committed PMC pass (profiles/pmc_insts.json)
    if os.path.exists(INSTS_FILE) and world == 1 and not fast:
        try:
            with open(INSTS_FILE) as f:
                pi = json.load(f)
            if pi.get("workload") == f"complex_{W}x{H}_s{s}_d{DEPTH}":
                n_valu = pi["sq_insts_valu_per_launch"]
                n_f64 = sum(pi.get(k, 0.) for k in ("sq_insts_valu_fma_f64_per_launch",
                                                    "sq_insts_valu_mul_f64_per_launch",
                                                    "sq_insts_valu_add_f64_per_launch",
                                                    "sq_insts_valu_trans_f64_per_launch"))
                simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
                # SIMD cycles the launch's VALU instructions occupy, over the SIMD-cycles available
                busy = VALU_CYCLES * (n_valu - n_f64) + VALU_CYCLES_F64 * n_f64
                avail = simds * GPU_CLOCK_HZ * (kms / 1e3)
                valu = {"insts_per_launch": n_valu, "f64_insts_per_launch": n_f64,
                        "achieved": round(n_valu / (kms / 1e3) / 1e9, 2),
                        "unit": "G wave-instr/s", "simd_busy_frac": round(busy / avail, 3),
                        "per_wave_segment": round(n_valu / max(1, st.segments / 64), 1),
                        "note": "simd_busy_frac = (2 cyc x f32/int + 4 cyc x f64 VALU instructions, PMC "
                                "SQ_INSTS_VALU*) / (SIMDs x clock x kernel time); profiles/pmc_insts.json "
                                "is from the profiled build"}
        except Exception:
            valu = None
    traffic = None
    if os.path.exists(PMC_FILE):
        try:
            with open(PMC_FILE) as f:
                pm = json.load(f)
            if pm.get("workload") == f"complex_{W}x{H}_s{s}_d{DEPTH}" and world == 1 and not fast:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = None
    if rank == 0:
        out = {
            "metric": "Msamples/sec (pixels\u00d7spp) on final-scene 1200\u00d7675 spp=500 d=50; CPU-ref speedup",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak" if weak else "strong",
            "vs_baseline": None,
            "dtype": "f32" if fast else "f64",
            "data": "synthetic (the reference's own procedural final scene, fixed seed)",
            "config": {"workload": f"complex_{W}x{H}_s{s}_d{DEPTH}", "width": W, "height": H,
                       "samples_sqrt": s, "spp": n_off, "max_depth": DEPTH,
                       "n_spheres": ns, "scene_seed": SEED, "render_seed": SEED, "frames": frames,
                       "parallelism": (f"frame-per-rank x{world} (render seed SEED+rank), no collective"
                                       if weak else f"row-cyclic x{world}" +
                                       (" + rccl all_gather" if world > 1 else "")),
                       "mode": ("fast_f32 (statistical parity; xoroshiro64** per (pixel, sample))"
                                if fast else "parity_f64 (bit-exact)")},
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                         "traffic": traffic,
                         "kernel": "rtw_fast_render" if fast else "rtw_render_persist (+ 7 small launches)",
                         "kernel_ms": round(kms, 3),
                         "algorithmic_flop_per_launch": brute_flop,
                         "executed_flop_per_launch": exec_flop,
                         "executed_tflops": round(executed, 3),
                         "executed_frac_of_fp32_peak": round(executed / FP32_VECTOR_PEAK, 4),
                         "note": ("fast mode: achieved = the same algorithmic brute-force work (segments x "
                                  "n_spheres x 17 FLOP) in f32 / kernel time, against the FP32 vector peak"
                                  if fast else None) or "achieved = SURVEY 8(d)'s algorithmic work (segments x n_spheres x 17 "
                                 "FLOP, the reference's f64 brute-force Scene::hit) / HIP-event kernel "
                                 "time, against the FP64 vector peak (parity mode is f64). The exact BVH "
                                 "and f32 filter reach that rate without executing it "
                                 "(executed_flop_per_launch: walk visits x 20 + exact f64 tests x 17), so "
                                 "frac is an effective rate, not pipe utilisation. What bounds the launch "
                                 "is VALU issue + latency of divergent per-lane work at 3 waves/SIMD "
                                 "(valu_issue.simd_busy_frac, DESIGN.md 4)",
                         "valu_issue": valu},
            "stats": {"accel": ["scan_f64", "scan_f32_filter", "bvh"][st.accel],
                      "node_visits_per_segment": round(st.node_visits / max(1, st.segments), 3),
                      "brute_segments": st.brute_segments, "lds_bytes": st.lds_bytes,
                      "parked_pixels": st.parked_pixels,
                      "segments": st.segments, "segments_per_sample": round(st.segments / max(1, st.samples), 4),
                      "lane_utilization": round(st.segments / max(1, 64 * st.wave_iterations), 4),
                      "exact_tests_per_segment": round(st.exact_tests / max(1, st.segments), 3),
                      "exact_wave_iters_per_wave_segment": round(st.exact_wave_iterations / max(1, st.wave_iterations), 3),
                      **({"walk_wave_iters_per_wave_iteration": round(st.exact_wave_iterations /
                                                                      max(1, st.wave_iterations), 3)}
                         if fast else {}),
                      "inside_cut_fraction": round(st.inside_segments / max(1, st.segments), 4),
                      "trap_skipped_fraction": round(st.trap_segments / max(1, st.segments), 4)},
        }
    if rank == 0 and world == 1 and a.e2e:
        out["end_to_end"] = end_to_end(cam.raw, sph, ns, mt, nm, s, render_seed, fast, kms)
    if rank == 0 and world == 1 and a.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cam.raw, sph, ns, mt, nm, s, a.cpu_row_stride)
        out["cpu_baseline"]["gpu_speedup"] = round(value / out["cpu_baseline"]["value"], 1)
        cl = out["cpu_baseline"]["clean_scheduler"]
        cl["gpu_speedup"] = round(value / cl["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    sess.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
