"""Forward attention throughput over shapes (HIP events), to separate tail / causal / sequence
effects:  python tools/attn_scan.py"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [  # B, H, HKV, S, hd, hdp, causal
    (4, 28, 4, 1536, 128, 128, True), (4, 28, 4, 1536, 128, 128, False), (16, 28, 4, 1536, 128, 128, True),
    (2, 28, 4, 4096, 128, 128, True), (2, 28, 4, 4096, 128, 128, False), (16, 16, 16, 729, 72, 96, False),
]


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


for B, H, HKV, S, hd, hdp, causal in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, H, S, hdp, device=dev, generator=g).bfloat16()
    k = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    v = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
    ms = timeit(lambda: ops.attn_fwd(q, k, v, hd, causal))
    fl = 4.0 * B * H * S * S * hd * (0.5 if causal else 1.0)
    print(json.dumps(dict(shape=[B, H, HKV, S, hd, causal], us=round(ms * 1e3, 1), tflops=round(fl / ms / 1e9, 1))), flush=True)
