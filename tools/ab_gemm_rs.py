"""A/B of the v8 GEMM's staging on the step's forward shapes: LDS-DMA (variant 16) vs register
staging (variant 22), interleaved runs, HIP events.   python tools/ab_gemm_rs.py [rounds]"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SHAPES = [  # name, M, N, K, act
    ("t.gate_up+swiglu", 6144, 37888, 3584, "swiglu"), ("t.lm_head", 6144, 152064, 3584, None),
    ("t.down", 6144, 3584, 18944, None), ("t.qkv", 6144, 4608, 3584, None), ("t.o", 6144, 3584, 3584, None),
    ("vit.fc1", 5832, 4304, 1152, "gelu_tanh"), ("vit.fc2", 5832, 1152, 4304, None), ("vit.qkv", 5832, 3456, 1152, None),
    ("s.gate_up+swiglu", 6144, 9728, 896, "swiglu"), ("s.lm_head", 6144, 151936, 896, None),
]
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
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


for name, M, N, K, act in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    it = max(3, int(2e12 / (2 * M * N * K)) + 3)
    best = {16: 1e30, 22: 1e30}
    for _ in range(rounds):
        for v in (16, 22):
            best[v] = min(best[v], timeit(lambda: ops.gemm(a, w, act=act, variant=v, split_k=1), it))
    fl = 2.0 * M * N * K
    print(json.dumps(dict(shape=name, us_dma=round(best[16], 1), us_rs=round(best[22], 1),
                          tf_dma=round(fl / best[16] / 1e6, 1), tf_rs=round(fl / best[22] / 1e6, 1),
                          gain=round(best[16] / best[22] - 1, 4))), flush=True)
