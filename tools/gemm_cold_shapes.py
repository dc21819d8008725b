"""kd_gemm (auto plan) on the step's big forward shapes in the step's cache state (1 GiB write before
each call; the activation re-written): median of iters calls.  For A/B of library builds / knobs:
    KDSTEP_LIB=... KD_...=... python tools/gemm_cold_shapes.py [iters]"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("KD_")) or "default"
res = []
for M, N, K in ((6144, 152064, 3584), (6144, 37888, 3584), (6144, 4608, 3584), (6144, 3584, 3584),
                (6144, 3584, 18944), (5832, 4304, 1152), (5832, 3456, 1152), (6144, 151936, 896)):
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    f = lambda: ops.gemm(a, w, out=out)
    f()
    ts = []
    for _ in range(it):
        junk.fill_(1.0)
        a.mul_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    res.append(f"{M}x{N}x{K} {ts[len(ts) // 2]:.1f}")
    del a, w, out
print(f"[{tag}] " + "  ".join(res), flush=True)
