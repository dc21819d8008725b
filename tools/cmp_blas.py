"""kd_gemm (auto plan, and each variant in KD_VARIANTS) vs torch.mm (hipBLASLt) on the KD step's GEMM shapes, interleaved in one process.
    python tools/cmp_blas.py [shapes.json] [top]
Shapes come from bench.py --shapes (default tools/step_shapes_c1.json); layouts:
  kk: C = A[M,K] . B[N,K]^T      kn: C = A[M,K] . W[K,N]      nn: C = A[K,M]^T . B[K,N]"""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else str(Path(__file__).resolve().parent / "step_shapes_c1.json")
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
VARS = [int(v) for v in os.environ.get("KD_VARIANTS", "16").split(",") if v]
rows = sorted(json.load(open(path)), key=lambda r: -r["total_ms"])[:top]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)


def timeit(f, it=10):
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
    return best



for r in rows:
    kind, shp = r["shape"].split(":")[:2]
    kind = kind.replace("_swiglu", "").replace("_dact", "")   # timed as the plain GEMM of that layout
    M, N, K = (int(x) for x in shp.split("x"))
    f32 = ":f32" in r["shape"]
    if kind == "gemm_kk":
        a = torch.randn(M, K, device=dev, generator=g).bfloat16(); b = torch.randn(N, K, device=dev, generator=g).bfloat16()
        mine = lambda v=0: ops.gemm(a, b, variant=v)
        ref = lambda: a @ b.t()
    elif kind == "gemm_kn":
        a = torch.randn(M, K, device=dev, generator=g).bfloat16(); w = torch.randn(K, N, device=dev, generator=g).bfloat16()
        mine = lambda v=0: ops.gemm(a, w.t(), variant=v)
        ref = lambda: a @ w
    else:
        a = torch.randn(K, M, device=dev, generator=g).bfloat16(); b = torch.randn(K, N, device=dev, generator=g).bfloat16()
        mine = lambda v=0: ops.gemm(a.t(), b.t(), out_dtype=torch.float32 if f32 else torch.bfloat16, variant=v)
        ref = lambda: a.t() @ b
    fl = 2.0 * M * N * K
    tm, tr = timeit(mine), timeit(ref)
    tv = {v: timeit(lambda: mine(v)) for v in VARS}
    extra = " ".join(f"| v{v} {t * 1e3:8.1f} us {fl / t / 1e9:7.1f} TF" for v, t in tv.items())
    print(f"{r['shape']:40s} kd {tm * 1e3:8.1f} us {fl / tm / 1e9:7.1f} TF {extra} | hipblaslt {tr * 1e3:8.1f} us "
          f"{fl / tr / 1e9:7.1f} TF", flush=True)
    del a
