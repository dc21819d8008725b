"""ORACLE — test infrastructure only, never the product path.

CPU restatement of the image half of the reference's collate_fn (DM:124-146: the HF
LlavaOnevision processor on the RGB / 3-channel depth uint8 images), i.e. transformers'
LlavaOnevisionImageProcessor (PIL backend) `_preprocess` for one image:
  get_image_patches    select_best_resolution -> _resize_for_patching (aspect-preserving,
                       get_patch_output_size) -> _pad_for_patching (centered zero pad) ->
                       divide_to_patches(384); plus the whole image resized to 384x384 first
  resize               PIL Image.resize(BICUBIC) of the uint8 RGB image
  rescale, normalize   float64(u8) * (1/255) -> float32; (x - 0.5) / 0.5 in float32
The bicubic resize is restated from Pillow's libImaging/Resample.c (precompute_coeffs,
normalize_coeffs_8bpc with PRECISION_BITS = 22, ImagingResampleInner's horizontal-then-vertical
8-bit passes with clip8); `resize_bicubic_u8` is checked against PIL itself
(tests/test_image.py) and the whole restatement against the installed processor's outputs
(tests/golden/image_*.npz, made by tests/golden/make_golden_image.py).  The pinned 4.45
processor is not installed: parity is pinned to transformers 5.15's PIL backend + Pillow 12.2.

Only tests/ may import this module.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 22
PATCH = 384
MEAN = STD = (0.5, 0.5, 0.5)


def bicubic_filter(x: float) -> float:
    """Resample.c bicubic_filter, a = -0.5."""
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def precompute_coeffs(in_size: int, out_size: int):
    """Resample.c precompute_coeffs (box = [0, in_size]) + normalize_coeffs_8bpc.
    Returns (ksize, bounds [out, 2] (xmin, count), kk int32 [out, ksize])."""
    support_f = 2.0
    scale = float(np.float32(in_size) - np.float32(0.0)) / out_size
    filterscale = max(scale, 1.0)
    support = support_f * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)   # C (int) truncates toward zero, like int()
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = [bicubic_filter((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for w in k:
            ww += w
        if ww != 0.0:
            k = [w / ww for w in k]
        for x, w in enumerate(k):
            kk[xx, x] = int(-0.5 + w * (1 << PRECISION_BITS)) if w < 0 else int(0.5 + w * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return ksize, bounds, kk


def _clip8(s: np.ndarray) -> np.ndarray:
    return np.clip(s >> PRECISION_BITS, 0, 255).astype(np.uint8)


def _pass(img: np.ndarray, out_size: int, axis: int) -> np.ndarray:
    """One 8-bit pass along `axis` (1 = horizontal, 0 = vertical) of an [H, W, C] uint8 image."""
    _, bounds, kk = precompute_coeffs(img.shape[axis], out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)            # [in, other, C]
    acc = np.full((out_size,) + src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
    for o in range(out_size):
        x0, n = bounds[o]
        acc[o] += np.tensordot(kk[o, :n], src[x0:x0 + n], axes=(0, 0))
    return np.moveaxis(_clip8(acc), 0, axis)


def resize_bicubic_u8(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """PIL Image.resize((out_w, out_h), BICUBIC) of an [H, W, C] uint8 image
    (ImagingResampleInner: horizontal pass first, each pass rounded to uint8)."""
    H, W = img.shape[:2]
    out = img
    if out_w != W:
        out = _pass(out, out_w, 1)
    if out_h != H:
        out = _pass(out, out_h, 0)
    return out.copy()


def select_best_resolution(original_size, possible_resolutions):
    oh, ow = original_size
    best, best_eff, best_waste = None, 0, float("inf")
    for h, w in possible_resolutions:
        scale = min(w / ow, h / oh)
        dw, dh = int(ow * scale), int(oh * scale)
        eff = min(dw * dh, ow * oh)
        waste = w * h - eff
        if eff > best_eff or (eff == best_eff and waste < best_waste):
            best, best_eff, best_waste = (h, w), eff, waste
    return best


def patch_output_size(h: int, w: int, th: int, tw: int):
    """transformers get_patch_output_size."""
    sw, sh = tw / w, th / h
    if sw < sh:
        return min(math.ceil(h * sw), th), tw
    return th, min(math.ceil(w * sh), tw)


PINPOINTS = [(h, w) for h in range(384, 2305, 384) for w in range(384, 2305, 384)]


def anyres_patches_u8(img: np.ndarray, pinpoints=PINPOINTS):
    """[H, W, 3] uint8 -> list of [3, 384, 384] uint8 patches (base image first)."""
    H, W = img.shape[:2]
    bh, bw = select_best_resolution((H, W), pinpoints)
    nh, nw = patch_output_size(H, W, bh, bw)
    resized = resize_bicubic_u8(img, nh, nw)
    py, px = (bh - nh) // 2, (bw - nw) // 2
    canvas = np.zeros((bh, bw, 3), np.uint8)
    canvas[py:py + nh, px:px + nw] = resized
    base = resize_bicubic_u8(img, PATCH, PATCH)
    tiles = [base] + [canvas[i:i + PATCH, j:j + PATCH] for i in range(0, bh, PATCH) for j in range(0, bw, PATCH)]
    return [t.transpose(2, 0, 1) for t in tiles]


def anyres_preprocess(img: np.ndarray, pinpoints=PINPOINTS) -> np.ndarray:
    """[H, W, 3] uint8 -> pixel_values [P, 3, 384, 384] float32 (one image of the processor)."""
    return np.stack([rescale_normalize_chw(p) for p in anyres_patches_u8(img, pinpoints)])


def rescale_normalize_chw(p: np.ndarray) -> np.ndarray:
    """rescale (float64 multiply by 1/255, cast to float32) then normalize ((x - mean) / std in
    float32) of a [3, h, w] uint8 patch."""
    x = (p.astype(np.float64) * (1 / 255)).astype(np.float32)
    mean = np.array(MEAN, np.float32)[:, None, None]
    std = np.array(STD, np.float32)[:, None, None]
    return (x - mean) / std
