"""v8n (variant 30, 256x128 tiles at two workgroups per CU) against the plan (variant 0) and v8
(variant 16, unsplit) on the step's forward shapes with their epilogues, in the step's cache state
(1 GiB write before each call): median of `iters` calls, us.
    python tools/v8n_ab.py [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)
SHAPES = [  # (name, M, N, K, epilogue)
    ("siglip qkv", 5832, 3456, 1152, "bias"), ("siglip o", 5832, 1152, 1152, "bias+res"),
    ("siglip fc1", 5832, 4304, 1152, "bias+gelu+aux"), ("siglip fc2", 5832, 1152, 4304, "bias+res"),
    ("student qkv", 6144, 1152, 896, "bias"), ("student o", 6144, 896, 896, "res"),
    ("student down", 6144, 896, 4864, "res"), ("projector 2", 5832, 896, 896, "bias"),
    ("teacher o", 6144, 3584, 3584, "res"), ("teacher down", 6144, 3584, 18944, "res")]
for name, M, N, K, epi in SHAPES:
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device=dev, generator=g).bfloat16() if "bias" in epi else None
    res = torch.randn(M, N, device=dev, generator=g).bfloat16() if "res" in epi else None
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if "aux" in epi else None
    act = "gelu_tanh" if "gelu" in epi else None
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    line = []
    for v in (0, 16, 30):
        f = lambda: ops.gemm(a, w, out=out, bias=bias, residual=res, aux=aux, act=act, variant=v,
                             split_k=1 if v in (16, 30) else 0)
        f()
        ts = []
        for _ in range(it):
            junk.fill_(1.0)
            a.mul_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        line.append(f"v{v} {ts[len(ts) // 2]:7.1f}")
    plan = ops.gemm_plan(a, w, out=out, bias=bias, residual=res, aux=aux, act=act)
    print(f"{name:13s} {M}x{N}x{K} {epi:14s} plan {plan}  " + "  ".join(line), flush=True)
