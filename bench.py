#!/usr/bin/env python3
"""Benchmark of the MI355X sampling path on BASELINE.json's headline workload.

Workload (BASELINE.json metric / configs[3]): the book's final random-spheres
scene (raytracing::complex, raytracing/mod.rs:54-126; 486 spheres at the fixed
scene seed), 1200x675, spp=500 -> samples_sqrt 23 (529 spp, the reference API
takes samples_sqrt), max_depth 50, f64 parity mode (bit-identical to the
reference restatement). One step = one whole-image render (Camera::threaded_render
equivalent, camera.rs:223-352) with the scene already resident in HBM.
`--size WxH --samples-sqrt S --depth D` select the other BASELINE configs
(config 3: --samples-sqrt 10; a config-5 rank: --size 4096x2304 --samples-sqrt 45
under torchrun --nproc-per-node 8).

N>1, BASELINE configs[3]'s scaling curve, two launch shapes, both row-cyclic
(row r -> GPU r % N) with the gather inside the timed step:
  * `python bench.py --gpus N` (one process): an rtw_group of N device entries
    (include/rtw_capi.h) -- one session and stream per GPU, the row tiles gathered
    on GPU 0 by one ncclGather over xGMI and un-permuted there. On a box with fewer
    than N GPUs the entries repeat the visible devices round-robin (the line then
    says "devices repeated; not a scaling point").
  * `torchrun --nproc-per-node N bench.py --gpus N` (one rank per GPU): each rank
    renders its rows, then an RCCL all_gather of the padded row tiles + un-permute
    (torch.distributed); `--scaling weak` renders one whole frame per rank instead
    (render seed SEED + rank, no collective).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size WxH] [--samples-sqrt S]
                    [--depth D] [--scaling strong|weak] [--mode parity|fast]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line (contract in the task statement). After the timed
region (N=1): the frame is hashed against the committed full-frame oracle
fixture when one exists (`parity`), the render kernel's counters are collected by
separate rocprofv3 --pmc passes of a one-frame child run (`roofline.valu_issue`,
`roofline.traffic`), the one-shot ABI call with host buffers + PPM is timed
(`end_to_end`), and the cpu_baseline leg times the C oracle (test infrastructure,
kind "port") on a bounded row sample of the same workload.
"""
from __future__ import annotations

import argparse
import csv
import glob
import hashlib
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

SEED = 1764892800000  # the package's DEFAULT_SEED (scene and render seed)
FLOP_PER_TEST = 17  # oc 3, half_b 5, c 6 (r*r hoisted), disc 3
FLOP_PER_VISIT = 20  # BVH walk step: slab test 6 FMA + 10 min/max, or the 17-FLOP sphere filter
FP32_VECTOR_PEAK = 157.3  # TFLOP/s, MI355X spec (MI355X_MICROARCH.md chip table)
FP64_VECTOR_PEAK = 78.6   # TFLOP/s, MI355X spec
HBM_PEAK = 8000.0         # GB/s (MI355X_MICROARCH.md)
GPU_CLOCK_HZ = 2.4e9      # MI355X peak engine clock (MI355X_MICROARCH.md)
SIMD_LANES = 32           # a SIMD issues 32 lanes per cycle: a wave64 f32/int op takes 2 cycles
MAIN_KERNEL = {"parity": "rtw_render_persist", "fast": "rtw_fast_render"}
PMC_FALLBACK = os.path.join(HERE, "profiles", "r06_pmc.json")  # stamped with the build id
# counter passes (never combined with tracing; FETCH_SIZE and WRITE_SIZE never share
# a pass: MI355X_MICROARCH.md, rocprofv3 block limits)
PMC_PASSES = {
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
    "insts": ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VALU_TRANS_F64",
              "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
              "SQ_INSTS_VALU_INT64"],
    "cycles": ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU",
               "SQ_ACTIVE_INST_ANY"],
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--size", default="1200x675", help="WxH")
    p.add_argument("--samples-sqrt", type=int, default=23)
    p.add_argument("--depth", type=int, default=50)
    p.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                   help="N>1: strong = the one frame row-cyclically sharded + RCCL all_gather "
                        "(BASELINE configs[3]); weak = one whole frame per rank (seed SEED+rank)")
    p.add_argument("--shard-of", default="",
                   help="N:r -- one process renders only rank r's rows of an N-rank strong split "
                        "(a rank of a multi-GPU config measured on one GPU; the other ranks are not run)")
    p.add_argument("--mode", choices=("parity", "fast"), default="parity",
                   help="parity = f64 bit-exact (the headline); fast = the f32 mode with "
                        "independent per-sample streams (statistical parity, tests/test_gpu_fast.py)")
    p.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the CPU leg")
    p.add_argument("--e2e", type=int, default=1,
                   help="0 disables the end-to-end leg (one-shot ABI call with host buffers + PPM)")
    p.add_argument("--pmc", type=int, default=1,
                   help="1: rocprofv3 --pmc passes of a one-frame child run (N=1, after the timed "
                        "region); 0: only the build-stamped profiles/r06_pmc.json")
    p.add_argument("--cpu-row-stride", type=int, default=0,
                   help="oracle renders every k-th row (0 = auto, ~10-30 s)")
    p.add_argument("--pmc-out", default="",
                   help="also write the live PMC summary (stamped with the build id) to this JSON file")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--pmc-shard", default="", help=argparse.SUPPRESS)  # N:r -- the child renders rank r's rows
    a = p.parse_args()
    a.width, a.height = (int(v) for v in a.size.lower().split("x"))
    a.sim = tuple(int(v) for v in a.shard_of.split(":")) if a.shard_of else None
    return a


def workload_name(a):
    return f"complex_{a.width}x{a.height}_s{a.samples_sqrt}_d{a.depth}"


# ----------------------------------------------------------------- PMC leg --
def pmc_child(a):
    """One frame of the workload through the one-shot ABI (the same launches as a
    bench step), run under rocprofv3 --pmc by pmc_live(); with --pmc-shard N:r only
    rank r's rows of the N-rank row-cyclic split (the shard that rank renders)."""
    import raytracing_in_a_weekend_rust_amd as rtw
    from raytracing_in_a_weekend_rust_amd import shard as sh
    cam, sph, ns, mt, nm = rtw.builtin_scene("complex", SEED, a.height, a.width, a.depth)
    one_shot = rtw.render_flat_fast if a.mode == "fast" else rtw.render_flat
    rows = None
    if a.pmc_shard:
        n, r = (int(v) for v in a.pmc_shard.split(":"))
        rows = sh.rows_of(r, n, a.height)
    one_shot(cam.raw, sph, ns, mt, nm, a.samples_sqrt, SEED, shard=rows)


def profiler_active():
    pre = os.environ.get("LD_PRELOAD", "") + os.environ.get("HSA_TOOLS_LIB", "")
    return "rocprof" in pre or any(k.startswith("ROCPROF") for k in os.environ)


def kernel_short_name(name):
    """The kernel's own identifier from a demangled rocprofv3 name: the last
    '::'-separated name before its template arguments / parameter list, e.g.
    'void rtw_fast::(anonymous namespace)::rtw_fast_render<true>(rtw_fast::FastParams)'
    -> 'rtw_fast_render', '(anonymous namespace)::rtw_seed_pixels((anonymous
    namespace)::KParams)' -> 'rtw_seed_pixels', '__amd_rocclr_copyBuffer' -> itself."""
    n = name.replace("(anonymous namespace)", "").strip()
    if n.startswith("void "):
        n = n[5:]
    cut = min([i for i in (n.find("<"), n.find("(")) if i >= 0], default=len(n))
    return n[:cut].split("::")[-1].strip() or name


def read_counters(d):
    """{kernel short name: {counter: per-dispatch mean}} from a rocprofv3 csv dir."""
    acc, disp = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                short = kernel_short_name(row["Kernel_Name"])
                c = row["Counter_Name"]
                k = (short, c)
                acc[k] = acc.get(k, 0.0) + float(row["Counter_Value"])
                disp.setdefault(k, set()).add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    out = {}
    for (short, c), v in acc.items():
        out.setdefault(short, {})[c] = v / max(1, len(disp[(short, c)]))
    return out


def pmc_live(a, timeout_s=75, shard=None):
    """Separate rocprofv3 --pmc passes over a one-frame child (no tracing in the same
    run; `shard` = (N, r): the child renders rank r's rows only). Returns
    {pass: {kernel: {counter: value per dispatch}}} or None."""
    exe = shutil.which("rocprofv3")
    if not exe or profiler_active():
        return None, "rocprofv3 not available" if not exe else "already under a profiler"
    tmp = tempfile.mkdtemp(prefix="rtw_pmc_")
    env = dict(os.environ, RTW_NO_TORCH="1", TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    res = {}
    try:
        for name, counters in PMC_PASSES.items():
            d = os.path.join(tmp, name)
            cmd = [exe, "--pmc", *counters, "-d", d, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-child", "--size", a.size,
                   "--samples-sqrt", str(a.samples_sqrt), "--depth", str(a.depth), "--mode", a.mode]
            if shard:
                cmd += ["--pmc-shard", f"{shard[0]}:{shard[1]}"]
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env,
                                 start_new_session=True, cwd=HERE)
            try:
                _, err = p.communicate(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.communicate()
                return (res or None), f"pass {name} timed out"
            if p.returncode != 0:
                return (res or None), f"pass {name} exited {p.returncode}: {err.decode()[-300:]}"
            res[name] = read_counters(d)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return res, "live"


def pmc_summary(res, kernel, build_id):
    """Per-launch values of the main kernel (+ write bytes of every kernel of the render)."""
    out = {"build_id": build_id, "kernel": kernel}
    k = lambda p: (res.get(p) or {}).get(kernel, {})  # noqa: E731
    if "FETCH_SIZE" in k("fetch") and "WRITE_SIZE" in k("write"):
        # FETCH_SIZE x2: gfx950 counts half of a wide streaming read (MI355X_MICROARCH.md
        # HBM section); both counters are in KB
        out["fetch_bytes"] = 2.0 * 1024.0 * k("fetch")["FETCH_SIZE"]
        out["write_bytes"] = 1024.0 * k("write")["WRITE_SIZE"]
        out["write_bytes_by_kernel"] = {kn: round(1024.0 * v["WRITE_SIZE"])
                                        for kn, v in res["write"].items() if "WRITE_SIZE" in v}
    for c, v in k("insts").items():
        out[c.lower()] = v
    for c, v in k("cycles").items():
        out[c.lower()] = v
    return out


def pmc_fallback(kernel, build_id):
    try:
        with open(PMC_FALLBACK) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/r06_pmc.json"
    if d.get("kernel") != kernel or d.get("workload") != "complex_1200x675_s23_d50":
        return None, "profiles/r06_pmc.json is for another kernel/workload"
    if d.get("build_id") != build_id:
        return None, f"profiles/r06_pmc.json is from build {d.get('build_id')}, library is {build_id}: refused"
    return d, "profiles/r06_pmc.json (same build id)"


# ------------------------------------------------------------ other legs --
def end_to_end(rtw, cam, sph, ns, mt, nm, s, seed, fast, kernel_ms, npix):
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
    samples = npix * (s * s if s else 1)
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


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), as SURVEY 8(d) asks."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(cam, sph, ns, mt, nm, s, stride, repeats=3):
    """Oracle (C restatement) on a row sample, ref-faithful scheduler: one job per
    pixel pulled by `threads` workers, dyn dispatch + Arc-refcount traffic as in
    camera.rs:269-292 / sphere.rs:69. Timed `repeats` times (the host's cores are
    shared, so single timings move by +-10 %): `value` is the median, `runs` every
    timing and `spread` (max - min) / median."""
    from oracle import oracle_ctypes as orc  # test infrastructure: checker/baseline only

    # the reference's own pool size on this host (not a cap of ours)
    threads, how = available_parallelism()
    if os.environ.get("RTW_CPU_THREADS"):
        threads, how = int(os.environ["RTW_CPU_THREADS"]), "RTW_CPU_THREADS override"
    if stride <= 0:  # ~2 rows per thread at the headline spp: ~6-8 s of CPU work per run
        work = cam.img_width * (s * s if s else 1) / (1200 * 529)
        stride = max(1, int(round(cam.img_height * work / (2 * threads))))
    n_rows = len(range(0, cam.img_height, stride))
    samples = n_rows * cam.img_width * (s * s if s else 1)
    runs = []
    for _ in range(max(1, repeats)):
        t0 = time.perf_counter()
        orc.render(cam, sph, ns, mt, nm, s, SEED, rows=(0, stride, n_rows), nthreads=threads, scheduler=0)
        runs.append(samples / (time.perf_counter() - t0) / 1e6)
    med = sorted(runs)[len(runs) // 2]
    # also the "clean" scheduler (rows pulled by the workers, direct
    # calls, no per-pixel job/refcount overhead), on the same sampled rows
    t0 = time.perf_counter()
    orc.render(cam, sph, ns, mt, nm, s, SEED, rows=(0, stride, n_rows), nthreads=threads, scheduler=1)
    c_dt = time.perf_counter() - t0
    return {"value": med, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"rows 0::{stride} ({n_rows} rows x {cam.img_width} px x {s * s} spp, "
                      f"{samples / 1e6:.1f} Msamples) of the same image, median of {len(runs)} runs "
                      f"({samples / med / 1e6:.1f} s each), ref-faithful per-pixel jobs, "
                      f"{os.cpu_count()} host cpus visible",
            "runs": [round(v, 4) for v in runs], "spread": round((max(runs) - min(runs)) / med, 4),
            "threads_rule": how, "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "clean_scheduler": {"value": samples / c_dt / 1e6, "unit": "Msamples/s", "cores": threads,
                                "sample": f"rows 0::{stride} ({n_rows} rows), {c_dt:.1f} s, row jobs, "
                                          "direct calls"}}


def parity_check(a, image, segments):
    """The timed frame against the committed oracle fixture, outside the timed region:
    the full-frame fixture (tests/golden/make_fullframe.py) when the workload has one,
    else its row sample (config 5: the sampled rows' SHA-256)."""
    if a.mode != "parity":
        return None
    full = os.path.join(HERE, "tests", "golden", f"fullframe_{workload_name(a)}.json")
    rows = os.path.join(HERE, "tests", "golden", f"rowsample_{workload_name(a)}.json")
    if os.path.exists(full):
        with open(full) as f:
            fix = json.load(f)
        fb = image.contiguous().cpu().numpy().astype("<f8", copy=False)
        ok = hashlib.sha256(fb.tobytes()).hexdigest() == fix["fb_sha256"]
        return {"fixture": os.path.relpath(full, HERE), "fb_sha256_ok": ok,
                "segments_ok": segments == fix["segments"], "segments": segments,
                "note": "last timed frame (gathered on rank 0 at N>1) vs the C oracle's full frame"}
    if os.path.exists(rows):
        with open(rows) as f:
            fix = json.load(f)
        fb = image.contiguous().cpu().numpy().astype("<f8", copy=False)
        bad = [y for y, h in zip(fix["rows"], fix["row_sha256"])
               if hashlib.sha256(fb[y].tobytes()).hexdigest() != h]
        return {"fixture": os.path.relpath(rows, HERE), "rows_checked": len(fix["rows"]),
                "rows_sha256_ok": not bad, "rows_differing": bad[:16], "segments": segments,
                "note": "last timed frame's sampled rows vs the C oracle's row sample "
                        "(the full frame is ~6 h of oracle time)"}
    return None


# ---------------------------------------------------------------- roofline --
def roofline(a, st, kms, main_ms, pm, pm_source, n_cu, grid):
    fast = a.mode == "fast"
    t = main_ms / 1e3
    brute_flop = st.sphere_tests * FLOP_PER_TEST
    if st.accel == 2:
        exec_flop = st.node_visits * FLOP_PER_VISIT + st.exact_tests * FLOP_PER_TEST
    else:
        exec_flop = brute_flop
    npix = st.pixels
    # SURVEY.md 8(d) algorithmic bytes: the framebuffer (24 B f64 / 12 B f32 a pixel)
    # + the scene staged once per workgroup (n_spheres x 32 B)
    alg_bytes = npix * (12 if fast else 24) + grid * st.sphere_tests // max(1, st.segments) * 32
    simds = 4 * n_cu
    peak_slots = simds * SIMD_LANES * GPU_CLOCK_HZ / 1e12  # T lane-slots/s (= 78.6 at 256 CUs)
    r = {"bound": "valu", "achieved": None, "peak": round(peak_slots, 2),
         "unit": "T VALU lane-slots/s", "frac": None, "traffic": None,
         "kernel": MAIN_KERNEL[a.mode], "kernel_ms": round(main_ms, 3),
         "render_ms": round(kms, 3),
         "algorithmic_bytes_per_launch": alg_bytes,
         "executed_flop_per_launch": exec_flop,
         "executed_tflops": round(exec_flop / t / 1e12, 3),
         "executed_frac_of_fp64_peak": round(exec_flop / t / 1e12 / FP64_VECTOR_PEAK, 4),
         "executed_frac_of_fp32_peak": round(exec_flop / t / 1e12 / FP32_VECTOR_PEAK, 4),
         "effective_bruteforce_tflops": round(brute_flop / t / 1e12, 3),
         "bruteforce_flop_per_launch": brute_flop,
         "pmc_source": pm_source,
         "note": "frac = VALU issue: lane-slots the main kernel's VALU instructions occupy "
                 "(PMC SQ_INSTS_VALU: 64 per wave64 f32/int op = 2 cycles of a 32-lane SIMD, "
                 "128 per f64 op = 4 cycles) / (SIMDs x 32 lanes x 2.4 GHz x kernel_ms). "
                 "executed_* = the work the BVH path runs (walk visits x 20 + exact f64 tests x "
                 "17 FLOP); effective_bruteforce_tflops = the reference's brute-force Scene::hit "
                 "work (segments x n_spheres x 17) over the same time, which the BVH does not "
                 "execute (SURVEY 8(f) row 4: reported apart). traffic = HBM bytes per launch "
                 "(PMC FETCH_SIZE x2 + WRITE_SIZE, separate passes)."}
    if pm and "sq_insts_valu" in pm:
        n_valu = pm["sq_insts_valu"]
        n_f64 = sum(pm.get(c, 0.) for c in ("sq_insts_valu_fma_f64", "sq_insts_valu_mul_f64",
                                            "sq_insts_valu_add_f64", "sq_insts_valu_trans_f64"))
        slots = 64.0 * (n_valu - n_f64) + 128.0 * n_f64
        ach = slots / t / 1e12
        r["achieved"] = round(ach, 3)
        r["frac"] = round(ach / peak_slots, 4)
        r["valu_issue"] = {"valu_insts_per_launch": n_valu, "f64_insts_per_launch": n_f64,
                           "salu_insts_per_launch": pm.get("sq_insts_salu"),
                           "lds_insts_per_launch": pm.get("sq_insts_lds"),
                           "valu_insts_per_wave_segment": round(n_valu / max(1, st.segments / 64), 1)}
        if pm.get("sq_wave_cycles"):
            r["valu_issue"]["wait_any_share"] = round(pm.get("sq_wait_any", 0.) / pm["sq_wave_cycles"], 4)
    if pm and "fetch_bytes" in pm:
        tr = pm["fetch_bytes"] + pm["write_bytes"]
        r["traffic"] = round(tr)
        r["traffic_detail"] = {"fetch_bytes": round(pm["fetch_bytes"]), "write_bytes": round(pm["write_bytes"]),
                               "traffic_over_algorithmic": round(tr / max(1, alg_bytes), 2),
                               "hbm_gbps": round(tr / t / 1e9, 2), "hbm_frac": round(tr / t / 1e9 / HBM_PEAK, 6),
                               "write_bytes_by_kernel": pm.get("write_bytes_by_kernel")}
    return r


def base_line(a, value, elapsed, n_gpus, frames, ns):
    fast = a.mode == "fast"
    W, H, s = a.width, a.height, a.samples_sqrt
    return {
        "metric": "Msamples/sec (pixels×spp) on final-scene 1200×675 spp=500 d=50; CPU-ref speedup",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": n_gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak" if a.scaling == "weak" else "strong",
        "vs_baseline": None,
        "dtype": "f32" if fast else "f64",
        "data": "synthetic (the reference's own procedural final scene, fixed seed)",
        "config": {"workload": workload_name(a), "width": W, "height": H,
                   "samples_sqrt": s, "spp": s * s if s else 1, "max_depth": a.depth,
                   "n_spheres": ns, "scene_seed": SEED, "render_seed": SEED, "frames": frames,
                   "mode": ("fast_f32 (statistical parity; xoroshiro64** per (pixel, sample))"
                            if fast else "parity_f64 (bit-exact)")},
    }


def group_main(a, torch, rtw, shard):
    """`python bench.py --gpus N` as a plain command: one process drives N device
    entries through an rtw_group (one session + stream per GPU, rows r -> entry
    r % N, ncclGather of the row tiles to GPU 0 + un-permute there, inside every
    timed step; rtw_group_render is blocking). Reference: camera.rs:253 -- the
    reference's pool takes every core of the machine from one call."""
    if a.scaling == "weak" or a.sim:
        raise SystemExit("--scaling weak / --shard-of run under torchrun (one rank per GPU)")
    visible = rtw.device_count()
    devs, repeated = shard.group_devices(a.gpus, visible)
    W, H, s = a.width, a.height, a.samples_sqrt
    cam, sph, ns, mt, nm = rtw.builtin_scene("complex", SEED, H, W, a.depth)
    fast = a.mode == "fast"
    g = rtw.Group(devs)
    g.set_scene(sph, ns, mt, nm)
    image = torch.empty((H, W, 3), dtype=torch.float32 if fast else torch.float64,
                        device=torch.device("cuda", devs[0]))
    render = g.render_fast if fast else g.render

    def sync_all():
        for d in sorted(set(devs)):
            torch.cuda.synchronize(d)

    for _ in range(a.warmup):
        render(cam.raw, s, SEED, image.data_ptr())
    sync_all()
    t0 = time.perf_counter()
    walls, roots = [], []
    for _ in range(a.steps):
        render(cam.raw, s, SEED, image.data_ptr())
        _, _, info = g.stats()
        walls.append(info["wall_ms"])
        roots.append(info["root_gather_ms"])
    sync_all()
    elapsed = time.perf_counter() - t0
    total, per, info = g.stats()
    value = W * H * (s * s if s else 1) * a.steps / elapsed / 1e6
    out = base_line(a, value, elapsed, a.gpus, 1, ns)
    out["config"]["parallelism"] = (
        f"one process, rtw_group of {a.gpus} entries on devices {devs}, row-cyclic, gather "
        f"{info['gather']} to device {devs[0]} + un-permute there"
        + (f" (RCCL fallback: {info['note']})" if info["fallback"] != "none" else "")
        + ("; devices repeated; not a scaling point" if repeated else ""))
    mains = [p.main_kernel_ms for p in per]
    out["group"] = {"devices": devs, "visible_devices": visible, "repeated": repeated,
                    "gather": info["gather"], "fallback": info["fallback"], "fallback_reason": info["note"],
                    "slowest_entry": max(range(len(mains)), key=mains.__getitem__),
                    "slowest_main_kernel_ms": round(max(mains), 3),
                    "main_kernel_ms_spread": round((max(mains) - min(mains)) / max(mains), 4) if max(mains) else 0.0,
                    "entry_kernel_ms": [round(p.kernel_ms, 3) for p in per],
                    "entry_main_kernel_ms": [round(p.main_kernel_ms, 3) for p in per],
                    "entry_pixels": [p.pixels for p in per],
                    "last_wall_ms": round(info["wall_ms"], 3),
                    "last_render_ms_max": round(info["render_ms_max"], 3),
                    "mean_root_gather_ms": round(sum(roots) / len(roots), 3),
                    "mean_wall_ms": round(sum(walls) / len(walls), 3),
                    "note": "root_gather_ms: GPU 0's stream from its own tile rendered to the image "
                            "complete (waiting for the slowest entry + gather + un-permute)"}
    # roofline of entry 0 (its rows of the split, its kernel time): the counter child
    # renders the same rows on device 0
    n_cu = torch.cuda.get_device_properties(devs[0]).multi_processor_count
    pm, pm_source = None, "not collected (--pmc 0)"
    if a.pmc and devs[0] == 0:
        res, why = pmc_live(a, shard=(len(devs), 0))
        kern = MAIN_KERNEL[a.mode]
        if res and "insts" in res and kern in res["insts"]:
            pm = pmc_summary(res, kern, rtw.build_id())
            pm_source = f"live rocprofv3 --pmc passes of a child run of entry 0's rows of the x{len(devs)} split"
        else:
            pm_source = f"live PMC failed ({why})"
    out["roofline"] = roofline(a, per[0], per[0].kernel_ms, per[0].main_kernel_ms, pm, pm_source, n_cu,
                               per[0].grid_blocks)
    out["roofline"]["scope"] = "entry 0 (device %d): its rows, its kernel time" % devs[0]
    out["parity"] = parity_check(a, image, total.segments)
    print(json.dumps(out), flush=True)
    g.close()


def main():
    a = parse()
    if a.pmc_child:
        pmc_child(a)
        return
    import torch  # first: librtw then shares torch's HIP runtime (same soname)
    import torch.distributed as dist

    import raytracing_in_a_weekend_rust_amd as rtw
    from raytracing_in_a_weekend_rust_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and a.gpus > 1:
        return group_main(a, torch, rtw, shard)
    if world != a.gpus and a.gpus > 1:
        raise SystemExit(f"--gpus {a.gpus} under a launcher of WORLD_SIZE {world}: one rank per GPU, "
                         "or drop the launcher (one process drives every GPU)")
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H, s, DEPTH = a.width, a.height, a.samples_sqrt, a.depth
    cam, sph, ns, mt, nm = rtw.builtin_scene("complex", SEED, H, W, DEPTH)
    n_off = s * s if s else 1
    weak = a.scaling == "weak"
    dev = torch.device("cuda", local)
    fast = a.mode == "fast"
    fdt = torch.float32 if fast else torch.float64
    sess = rtw.Session(local)
    sess.set_scene(sph, ns, mt, nm)
    if a.sim:  # rank r of an N-rank split, alone on this GPU
        if world > 1:
            raise SystemExit("--shard-of is a single-process measurement")
        plan = shard.StepPlan(a.sim[0], a.sim[1], H, W, False, SEED, fdt, dev, collective=False)
    else:
        plan = shard.StepPlan(world, rank, H, W, weak, SEED, fdt, dev)
    render = sess.render_fast if fast else sess.render
    stream = torch.cuda.current_stream(dev)
    kernel_ms = []

    def render_tile(pl):
        render(cam.raw, s, pl.render_seed, pl.tile.data_ptr(), stream=stream.cuda_stream, shard=pl.shard)

    def step(record):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        # the rank's rows, then (N>1 strong) the RCCL all_gather of the row tiles +
        # un-permute; ev1 between them brackets the render alone
        shard.step(plan, render_tile, after_render=lambda: ev1.record(stream))
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
    segments = st.segments
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        sg = torch.tensor([segments], dtype=torch.int64, device=dev)
        dist.all_reduce(sg, op=dist.ReduceOp.SUM)
        segments = int(sg.item()) if not weak else st.segments

    frames = world if weak else 1
    total_samples = frames * W * H * n_off * a.steps
    if a.sim:  # this rank's samples only
        total_samples = st.pixels * n_off * a.steps
    value = total_samples / elapsed / 1e6
    parity = parity_check(a, plan.image, segments) if rank == 0 and not a.sim else None

    out = None
    if rank == 0:
        pm, pm_source = None, "not collected (--pmc 0)"
        n_cu = torch.cuda.get_device_properties(local).multi_processor_count
        # the counter child renders what this rank rendered: the whole frame (N=1, or
        # weak scaling: rank 0's frame), or rank 0's rows of the strong split (the
        # other ranks wait at the final barrier meanwhile)
        child_shard = a.sim if a.sim else ((world, 0) if world > 1 and not weak else None)
        what = ("a one-frame child run" if child_shard is None else
                f"a child run of rank {child_shard[1]}'s rows of the x{child_shard[0]} split")
        if a.pmc:
            res, why = pmc_live(a, shard=child_shard)
            kern = MAIN_KERNEL[a.mode]
            if res and "insts" in res and kern in res["insts"]:
                pm, pm_source = pmc_summary(res, kern, rtw.build_id()), f"live rocprofv3 --pmc passes of {what} (this bench)"
                if a.pmc_out:
                    with open(a.pmc_out, "w") as f:
                        json.dump({**pm, "workload": workload_name(a), "mode": a.mode, "shard": child_shard}, f, indent=1)
            elif res and "insts" in res:  # the passes ran but matched no counters to the kernel
                seen = sorted({k for p in res.values() for k in p})
                pm_source = (f"live PMC passes ran but held no counters for kernel {kern} "
                             f"(kernels seen: {', '.join(seen[:8])}): frac/traffic not measured")
            else:
                pm_source = f"live PMC failed ({why})"
        if pm is None and a.mode == "parity" and workload_name(a) == "complex_1200x675_s23_d50" and child_shard is None:
            pm, fb_why = pmc_fallback(MAIN_KERNEL[a.mode], rtw.build_id())
            pm_source = (pm_source + "; " if a.pmc else "") + fb_why
        out = base_line(a, value, elapsed, world, frames, ns)
        out["config"]["parallelism"] = (f"rank {a.sim[1]} of a row-cyclic x{a.sim[0]} split, alone on one "
                                        "GPU (value = this rank's samples / its time; the other ranks "
                                        "not run)" if a.sim else plan.describe())
        out.update({
            "roofline": roofline(a, st, kms, st.main_kernel_ms or kms, pm, pm_source, n_cu, st.grid_blocks),
            "parity": parity,
            "build_id": rtw.build_id(),
            "stats": {"accel": ["scan_f64", "scan_f32_filter", "bvh"][st.accel],
                      "rank0_pixels": st.pixels,
                      "node_visits_per_segment": round(st.node_visits / max(1, st.segments), 3),
                      "brute_segments": st.brute_segments, "lds_bytes": st.lds_bytes,
                      "parked_pixels": st.parked_pixels,
                      "segments": st.segments, "segments_per_sample": round(st.segments / max(1, st.samples), 4),
                      "lane_utilization": round(st.segments / max(1, 64 * st.wave_iterations), 4),
                      "exact_tests_per_segment": round(st.exact_tests / max(1, st.segments), 3),
                      "exact_wave_iters_per_wave_segment": round(st.exact_wave_iterations / max(1, st.wave_iterations), 3),
                      "inside_cut_fraction": round(st.inside_segments / max(1, st.segments), 4),
                      "trap_skipped_fraction": round(st.trap_segments / max(1, st.segments), 4)},
        })
        if world == 1 and a.e2e:
            out["end_to_end"] = end_to_end(rtw, cam.raw, sph, ns, mt, nm, s, plan.render_seed, fast, kms, W * H)
        if world == 1 and a.cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cam.raw, sph, ns, mt, nm, s, a.cpu_row_stride)
            out["cpu_baseline"]["gpu_speedup"] = round(value / out["cpu_baseline"]["value"], 1)
            cl = out["cpu_baseline"]["clean_scheduler"]
            cl["gpu_speedup"] = round(value / cl["value"], 1)
        print(json.dumps(out), flush=True)
    sess.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
