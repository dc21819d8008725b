"""A/B of attention forward variants (KD_ATTN_FWD_V) on the KD step's shapes, HIP events, alternating.
    python tools/ab_attn_fwd.py [variants, default "0 64"]"""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

variants = sys.argv[1].split() if len(sys.argv) > 1 else ["0", "64"]
SHAPES = [("teacher.lm", 4, 28, 4, 1536, 128, 128, True), ("student.lm", 4, 14, 2, 1536, 64, 64, True),
          ("siglip", 8, 16, 16, 729, 72, 96, False)]
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


for name, B, H, HKV, S, hd, hdp, causal in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, H, S, hdp, device=dev, generator=g).bfloat16()
    k = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    v = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    fl = 4.0 * B * H * S * S * hd * (0.5 if causal else 1.0)
    res = {}
    for rep in range(3):
        for var in variants:
            os.environ["KD_ATTN_FWD_V"] = var
            res.setdefault(var, []).append(timeit(lambda: ops.attn_fwd(q, k, v, hd, causal)))
    os.environ.pop("KD_ATTN_FWD_V", None)
    print(json.dumps({"name": name, **{f"v{v_}_us": round(min(t), 1) for v_, t in res.items()},
                      **{f"v{v_}_tflops": round(fl / min(t) / 1e6, 1) for v_, t in res.items()}}), flush=True)
