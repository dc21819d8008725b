"""Micro-benchmark of kd_gemm on the step's GEMM shapes (bf16, random operands).

torch.matmul (hipBLASLt) is timed beside it only as a yardstick; it is never used by
the product path.  Usage: python tools/bench_gemm.py [--iters 20]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

# (name, M, N, K, layout) for B=4, L=1536 (M=6144) teacher / student
SHAPES = [
    ("t.qkv", 6144, 4608, 3584, "nt"), ("t.o", 6144, 3584, 3584, "nt"),
    ("t.gate_up", 6144, 37888, 3584, "nt"), ("t.down", 6144, 3584, 18944, "nt"),
    ("t.lm_head", 6144, 152064, 3584, "nt"),
    ("vit.qkv", 5832, 3456, 1152, "nt"), ("vit.fc1", 5832, 4304, 1152, "nt"), ("vit.fc2", 5832, 1152, 4304, "nt"),
    ("s.gate_up", 6144, 9728, 896, "nt"), ("s.lm_head", 6144, 151936, 896, "nt"),
    ("s.lm_head.dgrad", 6144, 896, 151936, "nn"), ("s.lm_head.wgrad", 151936, 896, 6144, "tn"),
    ("s.down.wgrad", 896, 4864, 6144, "tn"),
]


def run(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    rows = []
    for name, M, N, K, lay in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        if lay == "nt":
            A = torch.randn(M, K, device=dev, generator=g).bfloat16(); B = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
            f = lambda: ops.gemm(A, B)
            t = lambda: torch.matmul(A, B.t())
        elif lay == "nn":   # dX = dY W: A [M,K], W [K_out=K, N] -> B = W.t()
            A = torch.randn(M, K, device=dev, generator=g).bfloat16(); W = (torch.randn(K, N, device=dev, generator=g) * 0.05).bfloat16()
            f = lambda: ops.gemm(A, W.t())
            t = lambda: torch.matmul(A, W)
        else:               # dW = dY^T X : dY [K, M], X [K, N]
            dY = torch.randn(K, M, device=dev, generator=g).bfloat16(); X = torch.randn(K, N, device=dev, generator=g).bfloat16()
            f = lambda: ops.gemm(dY.t(), X.t(), out_dtype=torch.float32)
            t = lambda: torch.matmul(dY.t(), X)
        ms = run(f, a.iters)
        mt = run(t, a.iters)
        fl = 2.0 * M * N * K
        rows.append(dict(name=name, M=M, N=N, K=K, ms=round(ms, 4), tflops=round(fl / ms / 1e9, 1),
                         torch_ms=round(mt, 4), torch_tflops=round(fl / mt / 1e9, 1)))
        print(json.dumps(rows[-1]), flush=True)
        del f, t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
