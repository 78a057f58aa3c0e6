"""The statistical gate of the f32 fast mode, on 8-bit PPM values
(color.rs:196-247: (c^(1/2.2) * 255) as u64):
  * bias: per channel, |image mean of (fast - ref)| <= BIAS_TOL;
  * pixels: >= PIXEL_FRAC of the pixels have every channel within
    max(PIXEL_FLOOR, PIXEL_SIGMAS * sigma_MC) of the reference.
sigma_MC is the per-pixel standard deviation over independent f64 renders at the
same spp, taken as the maximum over the pixel's 3x3 neighbourhood: at a few spp
the 8-bit outcomes of a pixel are discrete and heavy-tailed (a sphere edge hit
by 1 sample in 9), and 8 renders often all miss the rare outcome (sigma = 0).
The pooled estimate passes the oracle against itself at >= 99.7%
(tests/test_fast_gate.py), the raw one only at ~95%."""
import numpy as np
from scipy.ndimage import maximum_filter

BIAS_TOL = 1.0      # 8-bit units, image mean per channel
PIXEL_FLOOR = 8.0   # 8-bit units
PIXEL_SIGMAS = 4.0
PIXEL_FRAC = 0.99


def to8(fb):
    """Color::gamma_correct + `as u64` (saturating, NaN -> 0), as floats."""
    x = np.nan_to_num(np.asarray(fb, dtype=np.float64), nan=0.0)
    return np.floor(np.power(np.maximum(x, 0.0), 1.0 / 2.2) * 255.0)


def gate(cand, ref, others):
    """(per-channel |bias|, fraction of pixels within tolerance) of cand vs ref;
    others: independent f64 renders for sigma_MC."""
    c8, r8 = to8(cand), to8(ref)
    sigma = np.std(np.stack([to8(o) for o in others]), axis=0, ddof=1)
    sigma = maximum_filter(sigma, size=(3, 3, 1), mode="nearest")
    bias = np.abs((c8 - r8).reshape(-1, 3).mean(axis=0))
    tol = np.maximum(PIXEL_FLOOR, PIXEL_SIGMAS * sigma)
    within = float((np.abs(c8 - r8) <= tol).all(axis=2).mean())
    return bias, within
