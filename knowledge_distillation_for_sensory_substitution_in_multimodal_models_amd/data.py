"""Synthetic batches in the layout of the reference's collate_fn (DM:97-167).

No dataset or processor is reachable offline, so batches are synthetic with the exact
tensor layout the hot path consumes:
  rgb_input_ids / depth_input_ids [B, L] int64 (same text for both, DM:127-150):
      24 random text ids + 1485 image tokens (151646) + 27 random text ids for 336x336
  rgb_pixel_values / depth_pixel_values [B, 2, 3, 384, 384] uniform in [-1, 1]
      (post-normalisation range), stored bf16
  image_sizes [B, 2] = (336, 336), kept host-side (metadata, read by the pack plan)
  labels = rgb input_ids with pad -> -100 (no padding here: equal lengths)
"""
from __future__ import annotations

import torch

from . import anyres
from .modeling import IMAGE_TOKEN_ID

TEXT_VOCAB = 151643


def synthetic_batch(B: int, device, L: int = 1536, image_hw=(336, 336), seed: int = 0,
                    pixel_dtype=torch.bfloat16, question_id: int = 0, cpu_rng: bool = False) -> dict:
    """cpu_rng=True draws the pixels on the CPU (bitwise identical across machines; tests),
    otherwise on the device (bench)."""
    n_img = anyres.num_image_tokens(image_hw)
    tiles = anyres.num_tiles(image_hw)
    if L < n_img + 2:
        raise ValueError(f"L={L} shorter than the {n_img} image tokens of a {image_hw} image")
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, TEXT_VOCAB, (B, L), generator=g, dtype=torch.int64)
    prefix = min(24, L - n_img - 1)
    ids[:, prefix:prefix + n_img] = IMAGE_TOKEN_ID
    rdev = "cpu" if cpu_rng else device
    gd = torch.Generator(device=rdev).manual_seed(seed + 1)
    rgb = (torch.rand(B, tiles, 3, 384, 384, generator=gd, device=rdev) * 2 - 1).to(pixel_dtype).to(device)
    depth = (torch.rand(B, tiles, 3, 384, 384, generator=gd, device=rdev) * 2 - 1).to(pixel_dtype).to(device)
    ids = ids.to(device)
    return {
        "rgb_input_ids": ids,
        "depth_input_ids": ids,
        "rgb_pixel_values": rgb,
        "depth_pixel_values": depth,
        "image_sizes": torch.tensor([list(image_hw)] * B, dtype=torch.int64),
        "labels": ids.clone(),
        "question_id": question_id,
    }
