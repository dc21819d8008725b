"""A/B of the norm forward (KD_NORM_FWD_V=1: previous kernel; default: k_norm_fwd2, loads hoisted) on
the step's shapes, HIP events, alternating.
    python tools/ab_norm_fwd.py"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
SHAPES = [("teacher rms bf16", 6144, 3584, True, False), ("siglip ln fp32", 5832, 1152, False, True),
          ("student rms fp32", 6144, 896, True, True)]


def timeit(f, it=50):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for name, R, D, rms, f32 in SHAPES:
    x = torch.randn(R, D, device=dev, generator=g)
    x = x if f32 else x.bfloat16()
    w = torch.randn(D, device=dev, generator=g).bfloat16()
    b = None if rms else torch.randn(D, device=dev, generator=g).bfloat16()
    y = torch.empty(R, D, dtype=torch.bfloat16, device=dev)
    nbytes = R * D * (4 if f32 else 2) + R * D * 2
    res = {}
    for rep in range(3):
        for v in ("1", "2"):
            os.environ["KD_NORM_FWD_V"] = v
            res.setdefault(v, []).append(timeit(lambda: ops.norm_fwd(x, w, b, 1e-6, rms=rms, out=y)))
    os.environ.pop("KD_NORM_FWD_V", None)
    old, new = min(res["1"]), min(res["2"])
    print(f"{name} {R}x{D}: previous {old:6.1f} us ({nbytes / old / 1e6:4.2f} TB/s)  hoisted {new:6.1f} us "
          f"({nbytes / new / 1e6:4.2f} TB/s)  {100 * (new / old - 1):+.1f}%", flush=True)
