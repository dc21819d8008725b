"""Host-side anyres packing plan of LLaVA-OneVision (index maps, no tensor math).

The reference reaches this through transformers (HF5 llava_onevision
`get_anyres_image_grid_shape` :152-182, `image_size_to_num_patches` :185-216,
`unpad_image` :219-256, `pack_image_features` :280-343; transformers
`select_best_resolution`).  Here it is restated as an index map: for each image token of
a sample, which (tile, patch) feature row it takes, or -1 for `image_newline`.  The map
depends only on image_sizes, is cached, uploaded once, and consumed on the device by
kd_image_src_map + kd_embed_assemble (no host sync in the step).
"""
from __future__ import annotations

import functools
import math

DEFAULT_PINPOINTS = tuple((h, w) for h in range(384, 2305, 384) for w in range(384, 2305, 384))
PATCH = 384          # vision_config.image_size: each anyres tile is 384x384
GRID = 27            # 384 // 14 patches per tile side
TOKENS_PER_TILE = GRID * GRID


def select_best_resolution(original_size, possible_resolutions):
    """Max effective resolution, then min wasted (transformers select_best_resolution)."""
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


def num_tiles(image_size, pinpoints=DEFAULT_PINPOINTS) -> int:
    """Base tile + grid tiles (HF5 image_size_to_num_patches)."""
    h, w = select_best_resolution(tuple(image_size), pinpoints)
    return (h // PATCH) * (w // PATCH) + 1


@functools.lru_cache(maxsize=256)
def pack_map(image_size: tuple, pinpoints=DEFAULT_PINPOINTS, max_patches: int = 9) -> tuple:
    """Sequence of (tile, patch) indices / -1 (newline) in the packed order of one image.

    Base tile first (729 rows), then the grid tiles laid out as one big
    (nph*27) x (npw*27) patch canvas, unpadded to the original aspect ratio, each canvas
    row followed by a newline token.
    """
    oh, ow = image_size
    bh, bw = select_best_resolution((oh, ow), pinpoints)
    nph, npw = bh // PATCH, bw // PATCH
    out = [(0, p) for p in range(TOKENS_PER_TILE)]
    H, W = nph * GRID, npw * GRID
    # unpad_image (HF5 :219-256): crop the canvas to the original aspect ratio
    r0, r1, c0, c1 = 0, H, 0, W
    if ow / oh > W / H:
        new_h = int(round(oh * (W / ow), 7))
        pad = (H - new_h) // 2
        r0, r1 = pad, H - pad
    else:
        new_w = int(round(ow * (H / oh), 7))
        pad = (W - new_w) // 2
        c0, c1 = pad, W - pad
    ch, cw = r1 - r0, c1 - c0
    if math.sqrt(ch * cw / (max_patches * GRID * GRID)) > 1.1:
        raise NotImplementedError("anyres_max_9 bilinear downsampling of very large grids is not supported")
    for R in range(r0, r1):
        ph, y = divmod(R, GRID)
        for Cc in range(c0, c1):
            pw, x = divmod(Cc, GRID)
            out.append((1 + ph * npw + pw, y * GRID + x))
        out.append(-1)
    return tuple(out)


def num_image_tokens(image_size, pinpoints=DEFAULT_PINPOINTS) -> int:
    return len(pack_map(tuple(image_size), pinpoints))


def batch_maps(image_sizes, tiles_per_sample: int):
    """Per-sample feature-row maps for a batch whose pixel_values are [B, P, 3, 384, 384].

    tiles_per_sample = P: feature rows are numbered over the flattened [B*P*729] vision
    output (a sample's tiles beyond num_tiles(image_size) are padding).  tiles_per_sample = 0:
    compact numbering over the REAL tiles only (sample b's rows follow sample b-1's
    num_tiles), what the reference's model runs through the vision tower (HF drops the
    padding tiles: pix_val[:num_patch]).  Returns (rows: list[list[int]], lengths: list[int]).
    """
    maps, lens = [], []
    base_tile = 0
    for b, hw in enumerate(image_sizes):
        m = pack_map(tuple(int(v) for v in hw))
        nt = num_tiles(hw)
        if tiles_per_sample and nt > tiles_per_sample:
            raise ValueError(f"sample {b}: image {tuple(hw)} needs {nt} tiles, batch has {tiles_per_sample}")
        base = (b * tiles_per_sample if tiles_per_sample else base_tile) * TOKENS_PER_TILE
        base_tile += nt
        maps.append([-1 if e == -1 else base + e[0] * TOKENS_PER_TILE + e[1] for e in m])
        lens.append(len(m))
    return maps, lens
