"""A/B of the fused q|k|v projection + head-major scatter (+ RoPE) epilogue (ops.gemm_qkv) across
GEMM builds: auto plan (0), v8 (24), v12 (26), on the step's three attention-input shapes.
Interleaved rounds in one process, HIP events, min over rounds.
    python tools/ab_qkv.py [--rounds 4] [--iters 10] [--variants 0,24,26]"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SHAPES = {  # B, S, K, nq, nkv, hd, hdp, rope
    "teacher": (4, 1536, 3584, 28, 4, 128, 128, True),
    "student": (4, 1536, 896, 14, 2, 64, 64, True),
    "siglip": (8, 729, 1152, 16, 16, 72, 96, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="0,24,26")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    vs = [int(v) for v in a.variants.split(",")]
    for name, (B, S, K, nq, nkv, hd, hdp, rope) in SHAPES.items():
        g = torch.Generator(device=dev).manual_seed(0)
        M, N = B * S, (nq + 2 * nkv) * hd
        x = torch.randn(M, K, generator=g, device=dev).bfloat16()
        w = (torch.randn(N, K, generator=g, device=dev) * K ** -0.5).bfloat16()
        bias = torch.randn(N, generator=g, device=dev).bfloat16()
        cos = sin = None
        if rope:
            inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float32, device=dev) / hd))
            f = torch.arange(S, dtype=torch.float32, device=dev)[:, None] * inv[None]
            cos, sin = f.cos().contiguous(), f.sin().contiguous()
        q = torch.empty((B, nq, S, hdp), dtype=torch.bfloat16, device=dev)
        k = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
        v = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        times = {}
        for r in range(a.rounds):
            for var in (vs if r % 2 == 0 else vs[::-1]):
                for kind in ("scatter", "plain"):
                    if kind == "scatter":
                        fn = lambda: ops.gemm_qkv(x, w, bias, q, k, v, S, nq, nkv, hd, hdp, cos, sin, variant=var)
                    else:
                        fn = lambda: ops.gemm(x, w, bias=bias, out=out, variant=var, split_k=1)
                    fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    times.setdefault(f"{kind}_v{var}_us", []).append(e0.elapsed_time(e1) / a.iters * 1e3)
        res = {k_: round(min(t), 1) for k_, t in times.items()}
        print(name, f"M={M} N={N} K={K}", json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
