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


PAD_ID = 151643   # <|endoftext|>, the Qwen2 tokenizer's pad token in the llava-onevision processors


def synthetic_batch_mixed(image_sizes, device, seed: int = 0, pixel_dtype=torch.bfloat16, prefix: int = 24,
                          suffix: int = 27, cpu_rng: bool = False, question_id: int = 0) -> dict:
    """A batch in the layout of the reference's collate_fn for real SUNRGBD geometry
    (DM:97-167, DS:185-212): one image per sample at its own size (480x640 -> 5 tiles and
    2,929 image tokens, SURVEY KAT 9; 336x336 -> 2 tiles, 1,485 tokens), `prefix` random
    text ids + the image tokens + `suffix` random text ids, right-padded with PAD_ID to the
    longest sample (processor padding=True), labels = ids with the pads -> -100 (DM:141-146),
    pixel_values [B, P_max, 3, 384, 384] with each sample's tiles past its own count zero
    (_pad_for_batching).  No attention mask (the reference passes none, DM:159-167)."""
    sizes = [tuple(int(v) for v in hw) for hw in image_sizes]
    B = len(sizes)
    lens = [prefix + anyres.num_image_tokens(hw) + suffix for hw in sizes]
    tiles = [anyres.num_tiles(hw) for hw in sizes]
    L, P = max(lens), max(tiles)
    g = torch.Generator().manual_seed(seed)
    ids = torch.full((B, L), PAD_ID, dtype=torch.int64)
    for b, hw in enumerate(sizes):
        n_img = anyres.num_image_tokens(hw)
        row = torch.randint(0, TEXT_VOCAB, (lens[b],), generator=g, dtype=torch.int64)
        row[prefix:prefix + n_img] = IMAGE_TOKEN_ID
        ids[b, :lens[b]] = row
    labels = torch.where(ids == PAD_ID, torch.full_like(ids, -100), ids)
    rdev = "cpu" if cpu_rng else device
    gd = torch.Generator(device=rdev).manual_seed(seed + 1)
    px = []
    for _ in range(2):   # rgb, depth
        t = torch.rand(B, P, 3, 384, 384, generator=gd, device=rdev) * 2 - 1
        for b in range(B):
            t[b, tiles[b]:] = 0
        px.append(t.to(pixel_dtype).to(device))
    ids = ids.to(device)
    return {
        "rgb_input_ids": ids,
        "depth_input_ids": ids,
        "rgb_pixel_values": px[0],
        "depth_pixel_values": px[1],
        "image_sizes": torch.tensor([list(hw) for hw in sizes], dtype=torch.int64),
        "labels": labels.to(device),
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


SIGLIP_MEAN = SIGLIP_STD = (0.5, 0.5, 0.5)   # image_mean / image_std of the llava-onevision-*-ov-hf checkpoints


def patch_output_size(h: int, w: int, th: int, tw: int):
    """transformers get_patch_output_size: aspect-preserving size inside (th, tw)."""
    import math
    sw, sh = tw / w, th / h
    if sw < sh:
        return min(math.ceil(h * sw), th), tw
    return th, min(math.ceil(w * sh), tw)


def process_images(images, device="cuda", image_mean=SIGLIP_MEAN, image_std=SIGLIP_STD,
                   dtype=torch.float32, patch: int = 384, pinpoints=anyres.DEFAULT_PINPOINTS) -> dict:
    """GPU counterpart of the image half of the processor call in the reference's collate_fn
    (DM:124-146; transformers LlavaOnevisionImageProcessor._preprocess): a list of [H, W, 3]
    uint8 images (numpy or tensors; RGB, or the 3-channel depth image) ->
    {"pixel_values": [B, P_max, 3, patch, patch] (dtype), "image_sizes": [B, 2] int64}.
    The plan (best pinpoint resolution, resize sizes) is host arithmetic on the image sizes;
    every pixel is computed by kd_image_resize_u8 / kd_anyres_tiles."""
    from . import ops
    ims = [(i if isinstance(i, torch.Tensor) else torch.from_numpy(i)).to(device, non_blocking=True) for i in images]
    plans = []
    for im in ims:
        if im.dtype != torch.uint8 or im.dim() != 3 or im.shape[2] != 3:
            raise RuntimeError(f"process_images: expected uint8 [H, W, 3], got {im.dtype} {tuple(im.shape)}")
        H, W = int(im.shape[0]), int(im.shape[1])
        bh, bw = anyres.select_best_resolution((H, W), pinpoints)
        plans.append((H, W, bh, bw, patch_output_size(H, W, bh, bw)))
    p_max = max(1 + (bh // patch) * (bw // patch) for _, _, bh, bw, _ in plans)
    pv = torch.empty((len(ims), p_max, 3, patch, patch), dtype=dtype, device=ims[0].device)
    for b, (im, (H, W, bh, bw, (nh, nw))) in enumerate(zip(ims, plans)):
        resized = ops.image_resize_u8(im, nh, nw)                    # _resize_for_patching
        base = ops.image_resize_u8(im, patch, patch)                 # resized_original_image
        ops.anyres_tiles(base, resized, (bh, bw), p_max, image_mean, image_std, dtype=dtype, patch=patch, out=pv[b])
    sizes = torch.tensor([[H, W] for H, W, *_ in plans], dtype=torch.int64)
    return {"pixel_values": pv, "image_sizes": sizes}
