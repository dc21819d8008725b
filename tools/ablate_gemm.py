"""A/B timing of the GEMM main-loop variants on one shape, interleaved rounds in one process.
    python tools/ablate_gemm.py [M N K]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (6144, 37888, 3584)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
a = torch.randn(M, K, device=dev, generator=g).bfloat16()
b = torch.randn(N, K, device=dev, generator=g).bfloat16()
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
names = {k: v for k, v in {5: "v3 (8 waves)", 16: "v8 (4 waves, AGPR acc)", 18: "v8 no DMA (ablation)",
                            19: "v8 L2-hot DMA (ablation)"}.items()
         if not __import__("os").environ.get("VARS") or str(k) in __import__("os").environ["VARS"].split(",")}
res = {v: [] for v in names}
for rnd in range(3):
    for v in names:
        f = lambda: ops.gemm(a, b, out=out, variant=v, split_k=1)
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 10)
fl = 2.0 * M * N * K
for v, n in names.items():
    t = min(res[v])
    print(f"{n:18s} {t:8.4f} ms {fl / t / 1e9:7.1f} TF/s  (rounds {[round(x, 4) for x in res[v]]})", flush=True)
