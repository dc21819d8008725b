"""Generate the image-preprocessing golden fixtures from transformers' own processor (dev container only).

    python tests/golden/make_golden_image.py

The reference's collate_fn (DM:124-146) runs the LLaVA-OneVision processor on each uint8 HxWx3
image (RGB, or the 3-channel depth image).  Its image half is LlavaOnevisionImageProcessor; the
installed transformers 5.15 runs it through the PIL backend (LlavaOnevisionImageProcessorPil,
torchvision is absent), Pillow 12.2.  This script runs that processor on seeded images and stores
its pixel_values losslessly: every output float is one of 256 values per channel (rescale +
normalize of a uint8), so the fixture holds the uint8 code of each output element plus the
processor's own 256-entry table per channel (computed by the same processor on a 0..255 ramp),
and checks that the decoding reproduces the processor output bit for bit before saving.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent

SIGLIP = dict(image_mean=[0.5, 0.5, 0.5], image_std=[0.5, 0.5, 0.5])  # the -ov-hf checkpoints' config
CLIP = dict(image_mean=[0.48145466, 0.4578275, 0.40821073], image_std=[0.26862954, 0.26130258, 0.27577711])


def images():
    g = np.random.default_rng(3)

    def smooth(h, w):
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
        base = np.stack([128 + 100 * np.sin(xx / (7 + 3 * c)) * np.cos(yy / (5 + 2 * c)) for c in range(3)], -1)
        return np.clip(base + g.normal(0, 12, base.shape), 0, 255).astype(np.uint8)

    return {
        "smooth_53x77": (smooth(53, 77), SIGLIP),
        "smooth_120x300": (smooth(120, 300), SIGLIP),
        "rand_200x150": (g.integers(0, 256, (200, 150, 3), dtype=np.uint8), SIGLIP),
        "smooth_64x64_clip": (smooth(64, 64), CLIP),
    }


def main():
    from transformers.models.llava_onevision.image_processing_pil_llava_onevision import (
        LlavaOnevisionImageProcessorPil)
    proc = LlavaOnevisionImageProcessorPil()
    for name, (img, norm) in images().items():
        pv = proc(images=[img], return_tensors="np", **norm)["pixel_values"][0]   # [P, 3, 384, 384] f32
        ramp = np.repeat(np.arange(256, dtype=np.uint8)[None, :, None], 3, axis=2)   # [1, 256, 3]
        lut = np.stack([proc.normalize(proc.rescale(ramp.transpose(2, 0, 1), 1 / 255), **{
            "mean": norm["image_mean"], "std": norm["image_std"]})[c, 0] for c in range(3)])  # [3, 256]
        codes = np.zeros(pv.shape, np.uint8)
        for c in range(3):
            order = np.argsort(lut[c])
            pos = np.searchsorted(lut[c][order], pv[:, c])
            codes[:, c] = order[np.clip(pos, 0, 255)]
            assert np.array_equal(lut[c][codes[:, c]], pv[:, c]), f"{name}: output not on the uint8 lattice"
        np.savez_compressed(HERE / f"image_{name}.npz", image=img, codes=codes, lut=lut.astype(np.float32),
                            mean=np.array(norm["image_mean"], np.float32), std=np.array(norm["image_std"], np.float32))
        print(f"{name}: {img.shape} -> pixel_values {pv.shape}")


if __name__ == "__main__":
    main()
