"""Build-time guard of KP()/CamRef (rtw_render.hip karg_base).

KP(field) reads KParams through the kernarg-segment pointer, which is the kernel's
own argument block only inside the kernel body (a noinline A/B build faulted with
hipErrorIllegalAddress in round 5). `make all` runs tools/check_karg.py on the device
listing; these tests check that the product listing passes it and that a build with
a deliberately outlined helper (RTW_KARG_SELFTEST: write_pixel noinline) fails it.
No GPU needed: hipcc cross-compiles the listing here.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import check_karg  # noqa: E402


def _listing():
    subprocess.run(["make", "-C", ROOT, "-s", "build/rtw_render.s"], check=True, capture_output=True,
                   timeout=600)
    return os.path.join(ROOT, "build", "rtw_render.s")


def test_product_listing_passes_guard():
    errors, report = check_karg.check(_listing())
    assert errors == [], errors
    names = " ".join(report)
    # the persistent kernel, the probe and the leftover launch all read KParams this way
    assert "rtw_render_persist" in names and "rtw_cost_probe" in names and "rtw_park_leftover" in names


def test_outlined_helper_fails_build():
    p = subprocess.run(["make", "-C", ROOT, "-s", "karg-selftest"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "violation detected as required" in p.stdout
    # the outlined write_pixel is named, and so are the kernels that now call it
    assert "write_pixel" in p.stdout and "makes calls" in p.stdout
