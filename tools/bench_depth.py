"""Time kd_depth_to_3ch (GPU convert_depth_image_into_3D, DS:64-112) on a SUNRGBD-sized batch and
report its HBM roofline; time the CPU oracle (numpy/scipy restatement of the reference) beside it.
    python tools/bench_depth.py [B] [H] [W]
Algorithmic bytes per pixel: read the uint16 depth sample once (2 B) + write 3 uint8 channels (3 B)."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H = int(sys.argv[2]) if len(sys.argv) > 2 else 530
W = int(sys.argv[3]) if len(sys.argv) > 3 else 730
dev = torch.device("cuda:0")
g = np.random.default_rng(0)
yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
base = 9000 + 20 * xx - 7 * yy + 2000 * np.sin(xx / 17.0) * np.cos(yy / 11.0)
imgs = np.stack([np.clip(base + g.normal(0, 30, (H, W)), 0, 65535) for _ in range(min(B, 8))]).astype(np.uint16)
imgs = np.concatenate([imgs] * ((B + len(imgs) - 1) // len(imgs)))[:B]
d = torch.from_numpy(imgs).to(dev)
out = torch.empty((B, H, W, 3), dtype=torch.uint8, device=dev)
f = lambda: ops.depth_to_3ch(d, out=out)  # noqa: E731
f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e30
for _ in range(5):
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) / 20)
alg = B * H * W * 5.0
print(f"depth_to_3ch B={B} {H}x{W}: {best * 1e3:.1f} us/batch = {B / best * 1e3:.0f} images/s; "
      f"algorithmic {alg / 1e6:.1f} MB -> {alg / best / 1e6:.0f} GB/s ({alg / best / 1e6 / 8000:.3f} of 8 TB/s)")
sys.path.insert(0, str(REPO))
from oracle import depth as D  # noqa: E402  (CPU baseline leg only)
t0 = time.perf_counter()
n = 0
while time.perf_counter() - t0 < 3.0:
    D.convert_depth_image_into_3D(imgs[n % len(imgs)])
    n += 1
cpu = (time.perf_counter() - t0) / n
print(f"cpu oracle (numpy/scipy, 1 thread): {cpu * 1e3:.1f} ms/image = {1 / cpu:.1f} images/s")
