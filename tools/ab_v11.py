"""A/B of the v11 GEMM (32x32x16 MFMAs, forced variant 23) against v8 (variant 24) on the
forward (K-major x K-major) shapes of the c1 step, interleaved rounds in one process, HIP
events; plus the fused gate|up + SwiGLU builds.

    python tools/ab_v11.py [--rounds 5] [--iters 10] [--variants 23,24]

(--variants 25: the wide-row DMA diagnostic build of v8, WRONG results: timing only.)
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SHAPES = [  # (name, M, N, K, act)
    ("t.gate_up+swiglu", 6144, 37888, 3584, "swiglu"), ("s.gate_up+swiglu", 6144, 9728, 896, "swiglu"),
    ("t.lm_head", 6144, 152064, 3584, None), ("t.qkv", 6144, 4608, 3584, None), ("t.o", 6144, 3584, 3584, None),
    ("t.down", 6144, 3584, 18944, None), ("vit.fc1", 5832, 4304, 1152, "gelu_tanh"), ("vit.qkv", 5832, 3456, 1152, None),
    ("vit.fc2", 5832, 1152, 4304, None), ("s.lm_head", 6144, 151936, 896, None),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--variants", default="23,24")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, M, N, K, act in SHAPES:
        if a.only and a.only not in name:
            continue
        x = (torch.randn(M, K, generator=g, device=dev)).bfloat16()
        w = (torch.randn(N, K, generator=g, device=dev) * K ** -0.5).bfloat16()
        out = torch.empty(M, N // 2 if act == "swiglu" else N, dtype=torch.bfloat16, device=dev)
        fl = 2.0 * M * N * K
        vs = [int(v) for v in a.variants.split(",")]
        times = {v: [] for v in vs}
        for r in range(a.rounds):
            for v in (vs if r % 2 == 0 else vs[::-1]):
                f = lambda: ops.gemm(x, w, out=out, act=act, variant=v, split_k=1)
                f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.iters * 1e3)
        res[name] = {f"v{v}_us": round(min(t), 1) for v, t in times.items()}
        res[name].update({f"v{v}_tflops": round(fl / min(t) / 1e6, 1) for v, t in times.items()})
        print(name, json.dumps(res[name]), flush=True)
        del x, w, out
    print(json.dumps(res))


if __name__ == "__main__":
    main()
