"""Run one attention forward shape repeatedly (for rocprofv3 PMC passes).
    python tools/attn_one.py teacher|student|siglip [iters] [bwd]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SH = {"teacher": (4, 28, 4, 1536, 128, 128, True), "student": (4, 14, 2, 1536, 64, 64, True),
      "siglip": (8, 16, 16, 729, 72, 96, False)}
B, H, HKV, S, hd, hdp, causal = SH[sys.argv[1]]
it = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B, H, S, hdp, device=dev, generator=g).bfloat16()
k = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
v = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
bwd = len(sys.argv) > 3 and sys.argv[3] == "bwd"
o, lse = ops.attn_fwd(q, k, v, hd, causal)
do = torch.randn(B, S, H, hd, device=dev, generator=g).bfloat16()
for _ in range(it):
    if bwd:
        ops.attn_bwd(q, k, v, o, do, lse, hd, causal)
    else:
        ops.attn_fwd(q, k, v, hd, causal)
torch.cuda.synchronize()
print("done")
