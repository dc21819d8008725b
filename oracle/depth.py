"""ORACLE — test infrastructure only, never the product path.

CPU restatement of the reference's depth -> 3-channel transform
  CustomSUNRGBDDatasetOneVision.convert_depth_image_into_3D
  (dataset/dataloader/OneVision/CustomSUNRGBDDatasetOneVision.py:64-112)
in numpy float32, with the reference's own third-party call kept for the filter
(scipy.ndimage.convolve with the Prewitt kernels, mode='reflect', DS:71-76, :97-98).
The image loading (PIL open + convert("I"), DS:86-87) is not restated: the input is the
int/float depth array that np.array(..., dtype=float32) produces from it.

Pinned against the reference itself: tests/golden/make_golden_depth.py imports the
reference dataset module in this container (its unavailable imports stubbed), runs its
convert_depth_image_into_3D on 16-bit PNGs it writes, and records inputs and outputs
(tests/golden/depth3_*.npz); tests/test_depth.py checks this file against them.

Only tests/ may import this module.

Note on channel 2: np.arctan2 in float32 is computed by numpy's SIMD library (SVML on
AVX-512 hosts), which is not correctly rounded; its last ulp depends on the host CPU.
`convert_depth_image_into_3D(..., return_float=True)` also returns the pre-truncation
values 255*(x - min)/(max - min) in float64 so tests can identify pixels whose uint8
depends on that ulp.
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import convolve

KX = np.array([[-1, 0, 1], [-1, 0, 1], [-1, 0, 1]], dtype=np.float32)   # DS:71-73
KY = np.array([[-1, -1, -1], [0, 0, 0], [1, 1, 1]], dtype=np.float32)   # DS:74-76


def _safe_normalize(arr: np.ndarray):
    """DS:79-83, float32 arithmetic as numpy>=2 evaluates it (NEP 50: python floats are weak)."""
    a_min, a_max = arr.min(), arr.max()
    if a_max == a_min:
        a_max = a_min + np.float32(1e-6)
    with np.errstate(invalid="ignore", divide="ignore"):
        q = np.float32(255.0) * (arr - a_min) / (a_max - a_min)
    return q, float(a_min), float(a_max)


def _to_u8(q: np.ndarray) -> np.ndarray:
    """ndarray.astype(np.uint8) of a float32 array as x86 numpy does it: truncate toward
    zero; NaN (0/0 when the 1e-6 fix-up rounds away) becomes 0."""
    q = np.where(np.isnan(q), np.float32(0), q)
    return q.astype(np.int64).astype(np.uint8)


def convert_depth_image_into_3D(depth: np.ndarray, return_float: bool = False):
    """depth [H, W] (any integer or float dtype) -> [H, W, 3] uint8 (DS:85-112)."""
    depth_array = np.asarray(depth).astype(np.float32)                   # DS:87
    q0, _, _ = _safe_normalize(depth_array)                               # DS:90-94 (same fix-up)
    depth_norm = _to_u8(q0)
    Gx = convolve(depth_norm.astype(np.float32), KX, mode="reflect")     # DS:97
    Gy = convolve(depth_norm.astype(np.float32), KY, mode="reflect")     # DS:98
    Gm = np.sqrt(Gx ** 2 + Gy ** 2)                                       # DS:101
    Gtheta = np.arctan2(Gy, Gx)                                           # DS:102
    q1, _, _ = _safe_normalize(Gm)                                        # DS:105
    q2, tlo, thi = _safe_normalize(Gtheta)                                # DS:106
    out = np.dstack([depth_norm, _to_u8(q1), _to_u8(q2)])                 # DS:109
    if not return_float:
        return out
    # float64 pre-truncation value of channel 2 from the correctly rounded angle
    th64 = np.arctan2(Gy.astype(np.float64), Gx.astype(np.float64))
    t_lo, t_hi = th64.min(), th64.max()
    den = (t_hi - t_lo) if t_hi != t_lo else 1e-6
    return out, 255.0 * (th64 - t_lo) / den


def prewitt_int(depth_norm: np.ndarray):
    """Integer Prewitt responses of a uint8 image under scipy's 'reflect' boundary, written
    out as the flipped-kernel sums (used by the tests to pin the boundary convention)."""
    d = np.pad(depth_norm.astype(np.int64), 1, mode="symmetric")
    H, W = depth_norm.shape
    win = lambda r, c: d[1 + r:1 + r + H, 1 + c:1 + c + W]  # noqa: E731
    gx = sum(win(r, -1) - win(r, 1) for r in (-1, 0, 1))
    gy = sum(win(-1, c) - win(1, c) for c in (-1, 0, 1))
    return gx, gy
