"""Developer tool: first-contact GPU check of librtw.so against the C oracle.
Prints parity results for small cases and a first timing of the final scene."""
import sys, time
import numpy as np
import raytracing_in_a_weekend_rust_amd as rtw
from oracle import oracle_ctypes as orc

seed = rtw.DEFAULT_SEED
print("devices", rtw.device_count(), flush=True)

# f64 sqrt / div correct rounding vs host
from raytracing_in_a_weekend_rust_amd import _capi as capi
import ctypes as C
rng = np.random.default_rng(1)
n = 1 << 20
a = np.abs(rng.standard_normal(n)) * 10.0 ** rng.integers(-30, 30, n)
b = rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)
osq = np.zeros(n); odiv = np.zeros(n)
P = C.POINTER(C.c_double)
capi.check(capi.lib.rtw_probe_f64_ops(0, a.ctypes.data_as(P), b.ctypes.data_as(P), n, osq.ctypes.data_as(P), odiv.ctypes.data_as(P)))
print("sqrt exact", np.array_equal(osq, np.sqrt(a)), "div exact", np.array_equal(odiv, a / b), flush=True)

# device seeds
out = (capi.U128 * 3000)()
capi.check(capi.lib.rtw_probe_device_seeds(0, capi.U128.of(seed), 123456, 3000, out))
print("device seeds", [out[i].value() for i in range(3000)] == rtw.seed_children(seed, 123456, 3000), flush=True)

def cmp(name, h, w, d, s, rows=None):
    cam, sph, ns, mt, nm = rtw.builtin_scene(name, seed, h, w, d)
    t = time.time(); fb, st = rtw.render_flat(cam.raw, sph, ns, mt, nm, s, seed, shard=rows); tg = time.time() - t
    t = time.time(); ref, seg = orc.render(cam.raw, sph, ns, mt, nm, s, seed, rows=rows); tc = time.time() - t
    eq = np.array_equal(fb, ref)
    nd = int((fb != ref).sum())
    print(f"{name} {w}x{h} s={s} d={d} rows={rows}: bitexact={eq} ndiff={nd} maxabs={np.abs(fb-ref).max():.3g} seg gpu={st.segments} cpu={seg} "
          f"kernel_ms={st.kernel_ms:.2f} gpu_wall={tg:.3f}s cpu={tc:.3f}s ppm_eq={rtw.format_ppm(fb)==orc.format_ppm(ref)}", flush=True)

cmp("three_lambertian", 225, 400, 8, 3)
cmp("complex", 36, 64, 50, 2)
cmp("simple", 90, 160, 25, 2)
cmp("complex", 90, 160, 50, 3)
cmp("complex", 675, 1200, 50, 2, rows=(7, 97, 7))

cam, sph, ns, mt, nm = rtw.builtin_scene("complex", seed, 675, 1200, 50)
for s in (10, 23):
    for rep in range(2):
        fb, st = rtw.render_flat(cam.raw, sph, ns, mt, nm, s, seed)
        ms = st.kernel_ms
        flop = st.sphere_tests * 17
        print(f"complex 1200x675 s={s}: kernel {ms:.1f} ms, {st.samples/ms/1e3:.1f} Msamples/s, seg/sample {st.segments/st.samples:.3f}, "
              f"lane util {st.segments/(64*st.wave_iterations):.3f}, {flop/ms/1e9:.2f} TFLOP/s alg", flush=True)
