"""Developer tool: kernel time per Scene::hit strategy on small grids (waves
mostly alone on their SIMD -> per-segment latency) and on the bench image."""
import os
os.environ.setdefault("RTW_AB", "1")  # the library reads tuning/diagnostic knobs only under RTW_AB
import sys

import raytracing_in_a_weekend_rust_amd as rtw

seed = rtw.DEFAULT_SEED
cases = [(36, 64, 2), (36, 64, 8), (90, 160, 4), (675, 1200, 4)]
for h, w, s in cases:
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", seed, h, w, 50)
    for mode in (1, 2):
        os.environ["RTW_ACCEL"] = str(mode)
        rtw.render_flat(cam.raw, sph, n, mt, nm, s, seed)
        fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, s, seed)
        print(f"{w}x{h} s={s} accel={st.accel}: kernel {st.kernel_ms:8.2f} ms  segments {st.segments}  "
              f"wave_iters {st.wave_iterations}  visits/seg {st.node_visits / max(1, st.segments):.1f}  "
              f"us/wave_iter(max-wave est) {st.kernel_ms * 1e3 / max(1, st.wave_iterations / max(1, st.grid_blocks * 4)):.2f}",
              flush=True)
