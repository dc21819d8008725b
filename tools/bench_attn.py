"""Time kd_attn_fwd / kd_attn_bwd on the KD step's attention shapes (HIP events).
    python tools/bench_attn.py"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SHAPES = [  # name, B, H, HKV, S, hd, hdp, causal
    ("teacher.lm", 4, 28, 4, 1536, 128, 128, True),
    ("student.lm", 4, 14, 2, 1536, 64, 64, True),
    ("siglip", 8, 16, 16, 729, 72, 96, False),
]
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
    return e0.elapsed_time(e1) / it


for name, B, H, HKV, S, hd, hdp, causal in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, H, S, hdp, device=dev, generator=g).bfloat16()
    k = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    v = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    o, lse = ops.attn_fwd(q, k, v, hd, causal)
    do = torch.randn(B, S, H, hd, device=dev, generator=g).bfloat16()
    f_ms = timeit(lambda: ops.attn_fwd(q, k, v, hd, causal))
    b_ms = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, hd, causal))
    frac = 0.5 if causal else 1.0
    fl = 4.0 * B * H * S * S * hd * frac           # QK^T + PV
    print(json.dumps(dict(name=name, fwd_ms=round(f_ms, 4), fwd_tflops=round(fl / f_ms / 1e9, 1),
                          bwd_ms=round(b_ms, 4), bwd_tflops_5mm=round(2.5 * fl / b_ms / 1e9, 1))), flush=True)
