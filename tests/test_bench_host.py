"""Host-side logic of bench.py and the group's RCCL fallback decision, on the CPU.

* `read_counters` must attribute rocprofv3 counter rows to the render kernels by
  their own names, whatever namespace / template decoration the demangled name
  carries (round 4's fast-mode line lost its roofline to a name match that took
  the namespace `rtw_fast` for the kernel). The two shapes are the ones the
  committed rocprof summaries hold (profiles/r04_v1/rocprof_kernel_stats_fast.csv,
  profiles/r04_v3/rocprof_kernel_stats.csv).
* `rtw_rccl_available` (include/rtw_capi.h) is the probe rtw_group_create uses to
  pick the RCCL gather or fall back to device copies; with RCCL made unloadable
  (RTW_RCCL_SONAME under RTW_AB) it must say no and why, without a GPU.
"""
import csv
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

FAST = "void rtw_fast::(anonymous namespace)::rtw_fast_render<true>(rtw_fast::FastParams)"
PERSIST = "void (anonymous namespace)::rtw_render_persist<true, 2, 768u, 64u>((anonymous namespace)::KParams)"
SEEDS = "(anonymous namespace)::rtw_seed_pixels((anonymous namespace)::KParams)"
PROBE = "void (anonymous namespace)::rtw_cost_probe<true>((anonymous namespace)::KParams)"


@pytest.mark.parametrize("name,short", [
    (FAST, "rtw_fast_render"), (PERSIST, "rtw_render_persist"), (SEEDS, "rtw_seed_pixels"),
    (PROBE, "rtw_cost_probe"), ("__amd_rocclr_copyBuffer", "__amd_rocclr_copyBuffer"),
    ("rtw_plain_kernel", "rtw_plain_kernel"),
])
def test_kernel_short_name(name, short):
    assert bench.kernel_short_name(name) == short


def test_committed_rocprof_summaries_name_the_main_kernels():
    for f, mode in (("profiles/r04_v1/rocprof_kernel_stats_fast.csv", "fast"),
                    ("profiles/r04_v3/rocprof_kernel_stats.csv", "parity")):
        with open(os.path.join(ROOT, f)) as fh:
            names = {bench.kernel_short_name(r["Name"]) for r in csv.DictReader(fh)}
        assert bench.MAIN_KERNEL[mode] in names, (f, names)


def _write_counters(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(w.fieldnames, r)))


@pytest.mark.parametrize("kernel,mode", [(FAST, "fast"), (PERSIST, "parity")])
def test_read_counters_and_summary_find_the_main_kernel(tmp_path, kernel, mode):
    """Two dispatches of the main kernel (per-dispatch mean) and one other kernel;
    the summary carries the main kernel's counters and every kernel's writes."""
    _write_counters(tmp_path / "insts", [
        (1, kernel, "SQ_INSTS_VALU", 100.0), (2, kernel, "SQ_INSTS_VALU", 300.0),
        (1, kernel, "SQ_INSTS_VALU_FMA_F64", 10.0), (2, kernel, "SQ_INSTS_VALU_FMA_F64", 30.0),
        (3, SEEDS, "SQ_INSTS_VALU", 7.0)])
    _write_counters(tmp_path / "fetch", [(1, kernel, "FETCH_SIZE", 4.0), (2, kernel, "FETCH_SIZE", 4.0)])
    _write_counters(tmp_path / "write", [(1, kernel, "WRITE_SIZE", 8.0), (3, SEEDS, "WRITE_SIZE", 2.0)])
    res = {p: bench.read_counters(str(tmp_path / p)) for p in ("insts", "fetch", "write")}
    main = bench.MAIN_KERNEL[mode]
    assert res["insts"][main]["SQ_INSTS_VALU"] == 200.0
    assert res["insts"]["rtw_seed_pixels"]["SQ_INSTS_VALU"] == 7.0
    pm = bench.pmc_summary(res, main, "test")
    assert pm["sq_insts_valu"] == 200.0 and pm["sq_insts_valu_fma_f64"] == 20.0
    assert pm["fetch_bytes"] == 2 * 1024 * 4.0 and pm["write_bytes"] == 1024 * 8.0
    assert pm["write_bytes_by_kernel"] == {main: 8192, "rtw_seed_pixels": 2048}


def test_cpu_baseline_threads_rule_is_reported():
    n, how = bench.available_parallelism()
    assert n >= 1 and "available_parallelism" in how


def _rccl_probe(env_extra):
    code = ("import raytracing_in_a_weekend_rust_amd as r; ok, why = r.rccl_available(); "
            "print(int(ok)); print(why)")
    env = dict(os.environ, RTW_NO_TORCH="1", **env_extra)
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    return lines[0] == "1", "\n".join(lines[1:])


def test_rccl_probe_reports_an_unloadable_rccl():
    """The group's fallback decision input: RCCL forced unloadable -> no, with the
    sonames tried in the reason (rtw_group_create then gathers by device copies and
    reports RTW_FALLBACK_NO_RCCL; only RTW_GROUP_RCCL_ALWAYS fails)."""
    ok, why = _rccl_probe({"RTW_AB": "1", "RTW_RCCL_SONAME": "librccl_missing_for_test.so"})
    assert not ok
    assert "librccl_missing_for_test.so" in why and "not loadable" in why


def test_rccl_soname_override_needs_the_ab_switch():
    """Production reads no tuning from the environment: without RTW_AB the override
    is ignored and the probe sees the real RCCL (present in this image)."""
    if not any(os.path.exists(os.path.join(d, "librccl.so.1")) for d in ("/opt/rocm/lib", "/opt/rocm/lib64")):
        pytest.skip("no librccl.so.1 in this image")
    ok, why = _rccl_probe({"RTW_AB": "0", "RTW_RCCL_SONAME": "librccl_missing_for_test.so"})
    assert ok, why
    assert why == ""
