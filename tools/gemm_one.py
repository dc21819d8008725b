"""Run one GEMM shape/variant repeatedly (for rocprofv3 PMC passes).
    python tools/gemm_one.py M N K [variant] [layout nt|nn|tn] [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

M, N, K = (int(x) for x in sys.argv[1:4])
var = int(sys.argv[4]) if len(sys.argv) > 4 else 0
lay = sys.argv[5] if len(sys.argv) > 5 else "nt"
it = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
if lay == "nt":
    A = torch.randn(M, K, device=dev, generator=g).bfloat16(); B = torch.randn(N, K, device=dev, generator=g).bfloat16()
    f = lambda: ops.gemm(A, B, variant=var)
elif lay == "nn":
    A = torch.randn(M, K, device=dev, generator=g).bfloat16(); W = torch.randn(K, N, device=dev, generator=g).bfloat16()
    f = lambda: ops.gemm(A, W.t(), variant=var)
else:
    dY = torch.randn(K, M, device=dev, generator=g).bfloat16(); X = torch.randn(K, N, device=dev, generator=g).bfloat16()
    f = lambda: ops.gemm(dY.t(), X.t(), out_dtype=torch.float32, variant=var)
for _ in range(it):
    f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    f()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / it
print(f"M={M} N={N} K={K} var={var} {lay}: {ms*1e3:.1f} us  {2*M*N*K/ms/1e9:.1f} TFLOP/s")
