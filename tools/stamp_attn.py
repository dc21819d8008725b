"""In-kernel stamps of the attention forward (KD_ATTN_FWD_V=34 build of k_attn_fwd32): where
each wave's cycles go. The stamps overwrite each wave's first row of a scratch Q copy.
    KD_ATTN_FWD_V=34 python tools/stamp_attn.py [B H HKV S hd hdp causal]"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

assert os.environ.get("KD_ATTN_FWD_V") == "34", "run with KD_ATTN_FWD_V=34"
B, H, HKV, S, hd, hdp, causal = (int(x) for x in sys.argv[1:8]) if len(sys.argv) > 7 else (4, 28, 4, 1536, 128, 128, 1)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
q0 = torch.randn(B, H, S, hdp, device=dev, generator=g).bfloat16()
k = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
v = torch.randn(B, HKV, S, hdp, device=dev, generator=g).bfloat16()
for _ in range(20):   # warm the clock
    q = q0.clone()
    ops.attn_fwd(q, k, v, hd, bool(causal))
torch.cuda.synchronize()
nqb = (S + 127) // 128
rows = q.view(B, H, S, hdp)[:, :, ::32, :].reshape(-1, hdp)          # every wave's first query row
st = rows.contiguous().view(torch.int32)[:, :8].cpu().double()        # [waves, 8]
st = st[: B * H * nqb * 4]
names = ["prologue", "tile compute", "tile wait+barrier", "epilogue", "total"]
tot = st[:, 4].mean().item()
print(f"B{B} H{H} HKV{HKV} S{S} hd{hd} causal{causal}: {st.shape[0]} waves, mean tiles/wg {st[:, 6].mean().item():.1f}, "
      f"computed/wave {st[:, 5].mean().item():.1f}")
for i, n in enumerate(names):
    col = st[:, i]
    print(f"  {n:18s} mean {col.mean().item():10.0f} ({100 * col.mean().item() / tot:5.1f}%)  p10 {col.quantile(0.1).item():9.0f}  p90 {col.quantile(0.9).item():9.0f}")
print(f"  shader clock {st[:, 4].sum().item() / st[:, 7].sum().item() * 0.1:.2f} GHz (s_memtime / s_memrealtime); "
      f"mean wave lifetime {st[:, 7].mean().item() / 100:.1f} us")
print(f"  compute per computed tile {st[:, 1].sum().item() / max(1.0, st[:, 5].sum().item()):.0f} cycles; "
      f"wait+barrier per tile {st[:, 2].sum().item() / st[:, 6].sum().item():.0f}")
