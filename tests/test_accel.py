"""Host self-check of the exact-result BVH walk (csrc/rtw_accel.h).

tools/accel_check.cpp (built by `make`, test infrastructure) runs the SAME walk
code the device kernel compiles against the reference's brute-force Scene::hit
(hittable.rs:131-143: every sphere, f64 Sphere::hit sphere.rs:39-71, first
minimum in index order) on camera/path rays, random rays and near-tangent rays,
and requires an identical (index, t-bits) result for every ray. No GPU needed.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "raytracing_in_a_weekend_rust_amd", "_lib", "accel_check")

SCENES = [
    ("complex", 1764892800000, 20000),
    ("complex", 1733400000000, 20000),
    ("simple", 1764892800000, 5000),
    ("three_lambertian", 1764892800000, 5000),
    ("threads", 1764892800000, 2000),
    ("super_simple", 1764892800000, 2000),
    ("random:40", 1, 20000),
    ("random:300", 2, 10000),
    ("random:700", 3, 5000),
    # near-tangent / overlapping clusters at offsets up to 2^13: inside-cut margins
    ("touch:30", 1, 10000),
    ("touch:100", 2, 10000),
    ("touch:200", 13, 10000),
    ("touch:150", 7, 10000),
]


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", ROOT, "-j8", "all"], check=True, capture_output=True)
    return EXE


# both candidate lists: the default device build's (0) and -DRTW_SELF_SKIP's (1)
@pytest.mark.parametrize("self_skip", [0, 1])
@pytest.mark.parametrize("scene,seed,paths", SCENES)
def test_walk_matches_scan(exe, scene, seed, paths, self_skip):
    if self_skip and not (scene.startswith("complex") or scene in ("random:300", "touch:100")):
        pytest.skip("self-skip variant: a representative subset")
    p = subprocess.run([exe, scene, str(seed), str(paths), str(self_skip)], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["bvh"], r
    assert r["mismatches"] == 0
    assert r["rays"] > paths
    assert r["early_miss"] > r["early_tests"] // 20, r  # sphere_early_miss was exercised
    if scene == "complex":
        # the walk replaces the 486-sphere scan by ~20 node/leaf tests
        assert r["visits_per_walk"] < 40, r
        assert r["fallbacks"] + r["overflows"] < r["rays"] // 1000, r
    assert (r["self_skips"] > 0) == bool(self_skip) or scene not in ("complex", "random:300"), r
    if scene == "complex" or scene.startswith("touch:"):
        assert r["inside_cuts"] > r["rays"] // 10, r  # the inside cut was exercised


def test_ineligible_scene_reports_no_bvh(exe):
    # > 16 huge spheres: the kernel keeps the filtered scan
    p = subprocess.run([exe, "random:1500", "5", "10"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0
    assert json.loads(p.stdout.strip())["bvh"] is False


def test_division_free_next01_exhaustive():
    """rtw_numeric.h's next01_of (the device's XorShift::next_01 tail, random.rs:40-52)
    equals the IEEE division m / 4294967295.0 for every m in [0, 2^32-2]."""
    exe = os.path.join(ROOT, "raytracing_in_a_weekend_rust_amd", "_lib", "next01_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "-j8", "all"], check=True, capture_output=True)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert json.loads(p.stdout)["mismatches"] == 0


def test_square_root_free_total_internal_reflection_test():
    """rtw_numeric.h's tir_exceeds (Dielectric::scatter's ratio * sqrt(1 - cos^2) > 1,
    materials.rs:94-98, decided from the squares away from the boundary) gives the
    reference's decision on 40M random, near-critical and edge inputs."""
    exe = os.path.join(ROOT, "raytracing_in_a_weekend_rust_amd", "_lib", "next01_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "-j8", "all"], check=True, capture_output=True)
    p = subprocess.run([exe, "tir", "20000000"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout)
    assert r["mismatches"] == 0 and r["tir_checked"] > 40_000_000


def test_trapped_path_replay_matches_serial_draws():
    """The drain groups' trapped-path replay (rtw_render.hip unit_vec_round: lane j of a
    64-lane round draws try j from T^(3j) of the base state, via rtw::try_table) yields
    the serial random_unit_vec loop's unit vectors (vec3.rs:219-232) and RNG states, in
    order, over 2000 random states x 70 vectors (host emulation of the device code)."""
    exe = os.path.join(ROOT, "raytracing_in_a_weekend_rust_amd", "_lib", "try_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "-j8", "all"], check=True, capture_output=True)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout)
    assert r["mismatches"] == 0 and r["checked"] == 140000
