"""Attention backward per call with the generic delta loop (KD_ATTN_DELTA_V=1) vs the unrolled
k_attn_delta_n, on the step's SigLIP and student LM shapes; HIP events, alternating."""
import os
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
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for name, B, H, HKV, S, hd, hdp, causal in (("siglip", 8, 16, 16, 729, 72, 96, False), ("student.lm", 4, 14, 2, 1536, 64, 64, True)):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, H, S, hdp, device=dev, generator=g).bfloat16()
    k = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    v = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    o, lse = ops.attn_fwd(q, k, v, hd, causal)
    do = torch.randn(B, S, H, hd, device=dev, generator=g).bfloat16()
    out = torch.empty(B * S, (H + 2 * HKV) * hd, dtype=torch.bfloat16, device=dev)
    res = {}
    for _ in range(3):
        for var in ("1", "2"):
            os.environ["KD_ATTN_DELTA_V"] = var
            res.setdefault(var, []).append(timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, hd, causal, dqkv=out)))
    os.environ.pop("KD_ATTN_DELTA_V", None)
    a, b_ = min(res["1"]), min(res["2"])
    print(f"{name}: backward with the delta loop {a:7.1f} us, unrolled delta {b_:7.1f} us ({b_ - a:+.1f} us)", flush=True)
