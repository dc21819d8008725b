"""Time the GPU image preprocessing (process_images: PIL-exact bicubic resizes + anyres tiles,
the processor call of collate_fn DM:124-146) on SUNRGBD-sized images, and the CPU oracle beside it.
    python tools/bench_image.py [B]
Algorithmic bytes per image: read the HxWx3 uint8 image twice (two resizes) + write P tiles of
3x384x384 bf16 (the layout the KD step consumes)."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import data  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
g = np.random.default_rng(0)
imgs = [torch.from_numpy(g.integers(0, 256, (530, 730, 3), dtype=np.uint8)).to(dev) for _ in range(B)]
f = lambda: data.process_images(imgs, device=dev, dtype=torch.bfloat16)  # noqa: E731
out = f()
torch.cuda.synchronize()
P = out["pixel_values"].shape[1]
best = 1e30
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    best = min(best, (time.perf_counter() - t0) / 10)
alg = B * (2 * 530 * 730 * 3 + P * 3 * 384 * 384 * 2)
print(f"process_images B={B} 530x730 -> [{B},{P},3,384,384] bf16: {best * 1e3:.2f} ms/batch (wall, incl. host "
      f"launch) = {B / best:.0f} images/s; {alg / best / 1e9:.0f} GB/s algorithmic")
from oracle import image as I  # noqa: E402  (CPU baseline leg only)
x = imgs[0].cpu().numpy()
t0 = time.perf_counter()
I.anyres_preprocess(x)
cpu = time.perf_counter() - t0
t0 = time.perf_counter()
from PIL import Image  # noqa: E402
im = Image.fromarray(x)
for _ in range(5):
    im.resize((384, 384), Image.BICUBIC)
    im.resize((1057, 768), Image.BICUBIC)
pil = (time.perf_counter() - t0) / 5
print(f"cpu: numpy oracle {cpu * 1e3:.0f} ms/image; PIL resizes alone {pil * 1e3:.1f} ms/image")
