"""Sweep kernel/tile (v3 256x256 / 256x128 / 128x256, v8 256x256 for K-major x K-major) x split-K for the KD step's GEMM shapes and
print the measured best next to the library's own plan (calibrates gemm.hip:plan_gemm).
    python tools/tune_gemm.py [shapes.json] [top]"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
src = sys.argv[1] if len(sys.argv) > 1 else None
top = int(sys.argv[2]) if len(sys.argv) > 2 else 60
if src:
    rows = json.load(open(src))[:top]
    shapes = [r["shape"] for r in rows]
else:
    shapes = ["gemm_nn:1152x1152x5832:f32:acc", "gemm_kn:6144x896x9728:bf16", "gemm_nn:151936x896x6144:f32:acc"]


def timeit(f, it=10):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


g = torch.Generator(device=dev).manual_seed(0)
for sh in shapes:
    parts = sh.split(":")
    kind, (M, N, K) = parts[0], map(int, parts[1].split("x"))
    f32 = parts[2] == "f32"
    acc = len(parts) > 3
    la, lb = kind[5], kind[6]
    a = torch.randn(K, M, device=dev, generator=g).bfloat16().t() if la == "n" else \
        torch.randn(M, K, device=dev, generator=g).bfloat16()
    b = torch.randn(K, N, device=dev, generator=g).bfloat16().t() if lb == "n" else \
        torch.randn(N, K, device=dev, generator=g).bfloat16()
    out = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    fl = 2.0 * M * N * K
    auto = timeit(lambda: ops.gemm(a, b, out=out, accumulate=acc))
    res = {}
    VARS = (5, 6, 7, 16, 20)
    for var in VARS:
        for sk in (1, 2, 3, 4, 6, 8, 12, 16):
            if sk > 1 and (K // 32) // sk < 4:
                continue
            if sk > 1 and sk * M * N * 4 > ops.GEMM_SPLITK_WS:
                continue
            res[(var, sk)] = timeit(lambda: ops.gemm(a, b, out=out, accumulate=acc, variant=var, split_k=sk))
    best = min(res, key=res.get)
    row = dict(shape=sh, auto_ms=round(auto, 4), auto_tf=round(fl / auto / 1e9, 1), best=list(best),
               best_ms=round(res[best], 4), best_tf=round(fl / res[best] / 1e9, 1),
               s1={v: round(res[(v, 1)], 4) for v in VARS},
               all={f"{v}/{s}": round(t, 4) for (v, s), t in sorted(res.items())})
    print(json.dumps(row), flush=True)
