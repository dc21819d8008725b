"""One GEMM shape timed per call with HIP events, warm (back-to-back) vs cold (a 1 GB write
between calls evicts the 256 MB Infinity Cache and the L2s) vs hot-chip (a large GEMM between
calls, so the timed GEMM runs at the clock the chip holds under a dense MFMA load).
    python tools/gemm_cold.py M N K [layout nt|nn|tn] [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

M, N, K = (int(x) for x in sys.argv[1:4])
lay = sys.argv[4] if len(sys.argv) > 4 else "nt"
it = int(sys.argv[5]) if len(sys.argv) > 5 else 20
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
if lay == "nt":
    A = torch.randn(M, K, device=dev, generator=g).bfloat16(); B = torch.randn(N, K, device=dev, generator=g).bfloat16()
    f = lambda: ops.gemm(A, B)
elif lay == "nn":
    A = torch.randn(M, K, device=dev, generator=g).bfloat16(); W = torch.randn(K, N, device=dev, generator=g).bfloat16()
    f = lambda: ops.gemm(A, W.t())
else:
    dY = torch.randn(K, M, device=dev, generator=g).bfloat16(); X = torch.randn(K, N, device=dev, generator=g).bfloat16()
    f = lambda: ops.gemm(dY.t(), X.t(), out_dtype=torch.float32)
junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)
BA = torch.randn(6144, 3584, device=dev, generator=g).bfloat16(); BB = torch.randn(18944, 3584, device=dev, generator=g).bfloat16()
big = lambda: ops.gemm(BA, BB)


def run(pre, name):
    ts = []
    for i in range(it):
        pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    print(f"{name:10s} M={M} N={N} K={K} {lay}: median {ts[len(ts) // 2]:.1f} us  min {ts[0]:.1f} "
          f"({2 * M * N * K / ts[len(ts) // 2] / 1e6:.0f} TFLOP/s at the median)", flush=True)


run(lambda: None, "warm")
run(lambda: junk.fill_(1.0), "cold")
run(big, "hot-chip")
run(lambda: (big(), junk.fill_(1.0)), "hot+cold")
