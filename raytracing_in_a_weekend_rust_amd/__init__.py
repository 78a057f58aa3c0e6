"""MI355X-native (gfx950 HIP) implementation of the per-pixel sampling hot path of
NicoElbers/Raytracing_in_a_weekend_rust (Camera::threaded_render -> ray_color ->
Scene::hit / Sphere::hit -> Material::scatter), behind the C ABI in
include/rtw_capi.h. See DESIGN.md."""
from ._capi import LIB_PATH, RtwError  # noqa: F401  (raises ImportError if librtw.so is missing)
from .api import (DEFAULT_SEED, Camera, Dielectric, Group, Lambertian, Metal, Scene,  # noqa: F401
                  SceneBuilder, Session, Sphere, build_id, builtin_scene, device_count, format_ppm,
                  rccl_available, render_flat, render_flat_fast, render_flat_multi, render_flat_multi_fast,
                  seed_children, shutdown, write_ppm, xorshift_next_01, xorshift_next_int)

__version__ = "0.7.0"
