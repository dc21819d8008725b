"""Cost of the lm_head GEMM's row-statistics epilogue (kd_gemm_desc.row_stats) in isolation:
the teacher / student lm_head shapes with and without it, interleaved rounds (HIP events).
    python tools/rst_cost.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


def timeit(f, it=5):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for name, M, N, K, top2 in (("teacher lm_head", 6144, 152064, 3584, True), ("student lm_head", 6144, 151936, 896, False)):
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    rs = torch.empty(M, (N + 255) // 256, 8, dtype=torch.float32, device=dev)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    best = {"plain": 1e30, "stats": 1e30}
    for _ in range(3):
        best["plain"] = min(best["plain"], timeit(lambda: ops.gemm(h, w, out=out, variant=16, split_k=1)))
        best["stats"] = min(best["stats"], timeit(lambda: ops.gemm(h, w, out=out, row_stats=rs, row_stats_vs=151936,
                                                                   row_stats_top2=top2)))
    print(f"{name}: plain {best['plain']:.1f} us, with row stats {best['stats']:.1f} us "
          f"(+{best['stats'] - best['plain']:.1f} us)", flush=True)
