"""Attention backward per call: head-major outputs + kd_qkv_merge vs the fused-gradient outputs
(kd_attn_bwd_desc.dqkv), on the step's SigLIP (MHA) and student LM (GQA + RoPE) shapes; HIP events."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


def timeit(f, it=20):
    for _ in range(3):
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
    return best * 1e3


for name, B, H, HKV, S, hd, hdp, causal, rope in (("siglip", 8, 16, 16, 729, 72, 96, False, False),
                                                   ("student.lm", 4, 14, 2, 1536, 64, 64, True, True)):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, H, S, hdp, device=dev, generator=g).bfloat16()
    k = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    v = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    o, lse = ops.attn_fwd(q, k, v, hd, causal)
    do = torch.randn(B, S, H, hd, device=dev, generator=g).bfloat16()
    cos = sin = None
    if rope:
        ang = torch.rand(S, hd // 2, device=dev, generator=g)
        cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    out = torch.empty(B * S, (H + 2 * HKV) * hd, dtype=torch.bfloat16, device=dev)

    def merged():
        dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, hd, causal)
        ops.qkv_merge(dq, dk, dv, B, S, H, HKV, hd, hdp, cos=cos, sin=sin, out=out)

    def direct():
        ops.attn_bwd(q, k, v, o, do, lse, hd, causal, dqkv=out, cos=cos, sin=sin)
    a, b_ = [], []
    for _ in range(3):
        a.append(timeit(merged))
        b_.append(timeit(direct))
    print(f"{name}: backward + merge {min(a):7.1f} us   fused-gradient outputs {min(b_):7.1f} us  ({100 * (min(b_) / min(a) - 1):+.1f}%)",
          flush=True)
