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


def convert_depth_image_into_3D(depth_image, device="cuda") -> torch.Tensor:
    """GPU counterpart of CustomSUNRGBDDatasetOneVision.convert_depth_image_into_3D
    (dataset/dataloader/OneVision/CustomSUNRGBDDatasetOneVision.py:64-112).

    `depth_image` is a path to the depth PNG (read as PIL mode "I", DS:86) or an [H, W]
    array / tensor of depth samples.  Returns the uint8 [H, W, 3] image (normalised depth,
    Prewitt magnitude, Prewitt angle) on `device` — what __getitem__ holds as
    `np.array(depth_image)` (DS:194-195).  Every pixel is computed by kd_depth_to_3ch."""
    from . import ops
    if isinstance(depth_image, (str, bytes)) or hasattr(depth_image, "__fspath__"):
        from PIL import Image
        import numpy as np
        depth_image = np.array(Image.open(depth_image).convert("I"))      # int32, DS:86
    t = depth_image if isinstance(depth_image, torch.Tensor) else torch.from_numpy(depth_image)
    if t.dtype not in (torch.uint16, torch.int32, torch.float32):
        t = t.to(torch.int32) if not t.is_floating_point() else t.to(torch.float32)
    return ops.depth_to_3ch(t.to(device, non_blocking=True))


def convert_depth_batch(depth_images, device="cuda") -> list:
    """A list of [H, W] depth maps (ragged sizes allowed) -> list of uint8 [H, W, 3] device
    tensors; maps of equal size share one batched launch."""
    from . import ops
    ts = [d if isinstance(d, torch.Tensor) else torch.from_numpy(d) for d in depth_images]
    out: list = [None] * len(ts)
    groups: dict = {}
    for i, t in enumerate(ts):
        groups.setdefault((tuple(t.shape), t.dtype), []).append(i)
    for (_, _), idx in groups.items():
        y = ops.depth_to_3ch(torch.stack([ts[i] for i in idx]).to(device, non_blocking=True))
        for k, i in enumerate(idx):
            out[i] = y[k]
    return out
