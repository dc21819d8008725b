"""A/B of v8 GEMM builds on the step's shapes: variant 16 (production) vs a forced variant
(22 register staging), interleaved runs, HIP events.
    python tools/ab_gemm_rs.py [rounds] [variant]"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SHAPES = [  # name, M, N, K, act, layout (nt forward, nn dgrad, tn wgrad)
    ("t.gate_up+swiglu", 6144, 37888, 3584, "swiglu", "nt"), ("t.lm_head", 6144, 152064, 3584, None, "nt"),
    ("t.down", 6144, 3584, 18944, None, "nt"), ("t.qkv", 6144, 4608, 3584, None, "nt"), ("t.o", 6144, 3584, 3584, None, "nt"),
    ("vit.fc1", 5832, 4304, 1152, "gelu_tanh", "nt"), ("vit.fc2", 5832, 1152, 4304, None, "nt"),
    ("vit.qkv", 5832, 3456, 1152, None, "nt"), ("s.gate_up+swiglu", 6144, 9728, 896, "swiglu", "nt"),
    ("s.lm_head", 6144, 151936, 896, None, "nt"), ("s.lm_head.dgrad", 6144, 896, 151936, None, "nn"),
    ("s.down.dgrad", 6144, 9728, 896, None, "nn"), ("s.lm_head.wgrad", 151936, 896, 6144, None, "tn"),
    ("vit.fc1.wgrad", 4304, 1152, 5832, None, "tn"),
]
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
VB = int(sys.argv[2]) if len(sys.argv) > 2 else 22
dev = torch.device("cuda:0")


def timeit(f, it):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for name, M, N, K, act, lay in SHAPES:
    if VB == 22 and lay != "nt":
        continue   # the register-staged build exists for K-major operands only
    g = torch.Generator(device=dev).manual_seed(0)
    if lay == "nt":
        a = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    elif lay == "nn":
        a = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(K, N, device=dev, generator=g) * 0.05).bfloat16().t()
    else:
        a = torch.randn(K, M, device=dev, generator=g).bfloat16().t()
        w = (torch.randn(K, N, device=dev, generator=g) * 0.05).bfloat16().t()
    it = max(3, int(2e12 / (2 * M * N * K)) + 3)
    best = {16: 1e30, VB: 1e30}
    for _ in range(rounds):
        for v in (16, VB):
            best[v] = min(best[v], timeit(lambda: ops.gemm(a, w, act=act, variant=v, split_k=1), it))
    fl = 2.0 * M * N * K
    print(json.dumps(dict(shape=name, us_v16=round(best[16], 1), **{f"us_v{VB}": round(best[VB], 1)},
                          tf_v16=round(fl / best[16] / 1e6, 1), **{f"tf_v{VB}": round(fl / best[VB] / 1e6, 1)},
                          gain=round(best[16] / best[VB] - 1, 4))), flush=True)
