"""Calibration of the fast-mode statistical gate (tests/fast_gate.py) on the CPU:
an f64 oracle render at another seed is a sample from the same distribution as
the reference, so it must pass the gate the f32 fast mode is held to
(tests/test_gpu_fast.py) -- the gate is not tighter than Monte Carlo noise."""
import raytracing_in_a_weekend_rust_amd as rtw
from oracle import oracle_ctypes as orc
from tests.fast_gate import BIAS_TOL, PIXEL_FRAC, gate

SEED = rtw.DEFAULT_SEED


def test_gate_passes_the_oracle_against_itself():
    cam, sph, n, mt, nm = rtw.builtin_scene("three_lambertian", SEED, 112, 200, 8)
    ref, _ = orc.render(cam.raw, sph, n, mt, nm, 3, SEED + 100)
    others = [orc.render(cam.raw, sph, n, mt, nm, 3, SEED + 101 + i)[0] for i in range(8)]
    for k in range(3):
        cand, _ = orc.render(cam.raw, sph, n, mt, nm, 3, SEED + 50 + k)
        bias, within = gate(cand, ref, others)
        assert (bias <= BIAS_TOL).all(), bias
        assert within >= PIXEL_FRAC, within
