"""Fused AdamW over the student's 893.6 M trainable parameters (c1): time per call and HBM rate
(30 B per parameter: fp32 master / m / v read + write, fp32 grad read, bf16 copy write).
    python tools/bench_adamw.py [n_params]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 893_585_216
dev = torch.device("cuda:0")
p = torch.randn(n, device=dev)
pb = p.bfloat16()
g = torch.randn(n, device=dev) * 1e-3
m = torch.zeros(n, device=dev)
v = torch.zeros(n, device=dev)
skip = torch.zeros(8, dtype=torch.int32, device=dev)
gs = torch.ones(1, device=dev)


def run(**kw):
    for i in range(3):
        ops.adamw(p, pb, g, m, v, 1e-5, 0.9, 0.999, 1e-8, 0.01, i + 1, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 10
    e0.record()
    for i in range(it):
        ops.adamw(p, pb, g, m, v, 1e-5, 0.9, 0.999, 1e-8, 0.01, i + 4, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    return ms, 30 * n / ms / 1e9


for name, kw in (("plain", {}), ("gscale + skip words", dict(gscale=gs, skip_words=skip))):
    ms, tbs = run(**kw)
    print(f"adamw n={n} {name:22s}: {ms:.3f} ms  {tbs:.2f} TB/s", flush=True)
