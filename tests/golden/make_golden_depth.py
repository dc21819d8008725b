"""Generate the depth-transform golden fixtures from the REFERENCE's own code (dev container only).

    python tests/golden/make_golden_depth.py

Imports dataset/dataloader/OneVision/CustomSUNRGBDDatasetOneVision.py from /root/reference.
Its module-level imports that are not installed here (torchvision, albumentations, llava) are
replaced by inert stub modules: convert_depth_image_into_3D (DS:64-112) uses none of them
(only PIL, numpy and scipy.ndimage.convolve).  The method is called unbound (it does not use
`self`) on 16-bit PNG files written here from seeded depth maps, exactly as __getitem__ calls it
(DS:194-195: np.array of the returned PIL image).  Only the input depth arrays and the
reference's uint8 outputs are committed (tests/golden/depth3_*.npz).
"""
from __future__ import annotations

import importlib.util
import sys
import tempfile
import types
from pathlib import Path
from unittest import mock

import numpy as np
from PIL import Image

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference")
DS_PATH = REF / "dataset/dataloader/OneVision/CustomSUNRGBDDatasetOneVision.py"


def _stub(name):
    m = types.ModuleType(name)
    m.__getattr__ = lambda attr: mock.MagicMock(name=f"{name}.{attr}")
    sys.modules[name] = m
    return m


def _load_reference():
    import transformers  # noqa: F401  (real package; imported before torchvision is stubbed)
    transformers.AutoProcessor  # noqa: B018
    for n in ["torchvision", "torchvision.transforms", "torchvision.transforms.functional", "albumentations",
              "llava", "llava.mm_utils", "llava.model", "llava.model.builder", "llava.constants",
              "llava.conversation"]:
        if n not in sys.modules:
            try:
                __import__(n)
            except ImportError:
                _stub(n)
    spec = importlib.util.spec_from_file_location("ref_ds_onevision", DS_PATH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.CustomSUNRGBDDatasetOneVision


def depth_maps():
    """Seeded depth maps covering the reference's cases: smooth scene-like 16-bit depth with
    noise and invalid (0) holes, odd/ragged sizes, thin images (reflect boundary on both sides),
    a flat image (the max == min fix-up) and a two-level step."""
    g = np.random.default_rng(7)
    out = {}
    H, W = 96, 128
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    scene = 8000 + 30 * xx + 12 * yy + 1500 * np.sin(xx / 9.0) * np.cos(yy / 13.0)
    scene += g.normal(0, 40, size=scene.shape)
    scene[g.random(scene.shape) < 0.03] = 0   # SUNRGBD invalid-depth holes
    out["scene_96x128"] = np.clip(scene, 0, 65535).astype(np.uint16)
    out["rand_53x77"] = g.integers(0, 65536, size=(53, 77), dtype=np.uint16)
    out["thin_1x40"] = g.integers(100, 5000, size=(1, 40), dtype=np.uint16)
    out["thin_37x2"] = g.integers(100, 5000, size=(37, 2), dtype=np.uint16)
    out["flat_16x24"] = np.full((16, 24), 4321, dtype=np.uint16)
    step = np.full((20, 30), 1000, dtype=np.uint16)
    step[:, 15:] = 3000
    out["step_20x30"] = step
    return out


def main():
    cls = _load_reference()
    tmp = Path(tempfile.mkdtemp(prefix="depth_golden_"))
    for name, d in depth_maps().items():
        path = tmp / f"{name}.png"
        Image.fromarray(d).save(path)            # 16-bit grayscale PNG, as SUNRGBD stores depth
        back = np.array(Image.open(path).convert("I"))
        assert np.array_equal(back, d.astype(np.int32)), name
        ref = np.array(cls.convert_depth_image_into_3D(None, str(path)))  # DS:194-195
        assert ref.dtype == np.uint8 and ref.shape == d.shape + (3,), (name, ref.shape)
        np.savez_compressed(HERE / f"depth3_{name}.npz", depth=d, out=ref)
        print(f"{name}: {d.shape} -> {ref.shape}, channel means {ref.reshape(-1, 3).mean(0).round(2)}")


if __name__ == "__main__":
    main()
