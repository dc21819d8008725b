"""Where the fused-gradient attention backward differs from backward + qkv_merge (diagnostic)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
for (B, H, HKV, S, hd) in [(2, 14, 2, 200, 64), (1, 4, 1, 130, 128)]:
    for rope in (False, True):
        g = torch.Generator(device=dev).manual_seed(7)
        q = torch.randn(B, H, S, hd, device=dev, generator=g).bfloat16()
        k = torch.randn(B, HKV, S, hd, device=dev, generator=g).bfloat16()
        v = torch.randn(B, HKV, S, hd, device=dev, generator=g).bfloat16()
        o, lse = ops.attn_fwd(q, k, v, hd, True)
        do = torch.randn(B, S, H, hd, device=dev, generator=g).bfloat16()
        cos = sin = None
        if rope:
            ang = torch.rand(S, hd // 2, device=dev, generator=g) * 6.0
            cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
        dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, hd, True)
        ref = ops.qkv_merge(dq, dk, dv, B, S, H, HKV, hd, hd, cos=cos, sin=sin)
        out = torch.full_like(ref, 3.0)
        ops.attn_bwd(q, k, v, o, do, lse, hd, True, dqkv=out, cos=cos, sin=sin)
        torch.cuda.synchronize()
        for name, a, b_ in (("dq", 0, H * hd), ("dk", H * hd, (H + HKV) * hd), ("dv", (H + HKV) * hd, (H + 2 * HKV) * hd)):
            x, y = out[:, a:b_].float(), ref[:, a:b_].float()
            bad = (out[:, a:b_] != ref[:, a:b_])
            nbad = int(bad.sum())
            col = bad.nonzero()[:, 1] % hd if nbad else torch.tensor([])
            print(f"B{B} H{H} HKV{HKV} S{S} hd{hd} rope={rope} {name}: mismatches {nbad}/{bad.numel()} "
                  f"max|diff| {float((x - y).abs().max()):.3e} rel {float(((x - y).abs() / (y.abs() + 1e-6)).max()):.2e} "
                  f"cols {sorted(set(col.tolist()))[:12]}", flush=True)
