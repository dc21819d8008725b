"""Cost of the LoCa override-column loads in the fused loss at the c1 shape: the same call with
random teacher logits (top-1 / top-2 spread over the vocabulary: thousands of override columns)
and with one dominant teacher column (top-1 the same in every row: a few hundred override columns).
    python tools/loss_ovr_cost.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

B, L, Vs, Vt = 4, 1536, 151936, 152064
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
s = (torch.randn(B, L, Vs, device=dev, generator=g) * 2).bfloat16()
t = (torch.randn(B, L, Vt, device=dev, generator=g) * 2).bfloat16()
lab = torch.full((B, L), 151646, dtype=torch.int64, device=dev)
lab[:, :24] = torch.randint(0, 151643, (B, 24), device=dev, generator=g)
lab[:, -27:] = torch.randint(0, 151643, (B, 27), device=dev, generator=g)


def timeit(f, it=5):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        for _ in range(it):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / it)
    return best * 1e3


for name in ("random teacher", "one dominant column"):
    if name != "random teacher":
        t[..., 7] = 40.0
        t[..., 11] = 30.0
    stats = torch.empty(0)
    us = timeit(lambda: ops.kd_loss_fwd_bwd(s, t, lab, "loca", temperature=1.0))
    ncols = torch.unique(torch.cat([lab.flatten(), t[..., :Vs].float().topk(2, dim=-1).indices.flatten()])).numel()
    print(f"{name:22s}: {us:7.0f} us per call, ~{ncols} distinct label / top-2 columns", flush=True)
