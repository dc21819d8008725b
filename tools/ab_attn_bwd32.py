"""A/B of the attention backward on the KD step's shapes: the product pair (the 32x32x16
k_attn_bwd_dq32 + the 16x16x32 k_attn_bwd_dkdv2), the round-6 16x16x32 pair (KD_ATTN_BWD_V=2) and the
all-32x32 pair (k_attn_bwd_dq32 + k_attn_bwd_dkdv32, KD_ATTN_BWD_V=32).

Runs against the A/B library (the only one that reads KD_ATTN_BWD_V):
    KDSTEP_LIB=tools/ab/libkdstep_ab.so python tools/ab_attn_bwd32.py
Per shape and arm: HIP-event time of kd_attn_bwd (20 calls after 3 warm-ups, min of 3 rounds) and
the worst element error of dq / dk / dv against a torch fp32 autograd reference on the same bf16
inputs, as a multiple of the tests' bound (8e-2 rms + 3e-2 |ref|; <= 1 passes).
"""
import json
import math
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SHAPES = [  # name, B, H, HKV, S, hd, hdp, causal
    ("student.lm", 4, 14, 2, 1536, 64, 64, True),
    ("siglip", 8, 16, 16, 729, 72, 96, False),
]
dev = torch.device("cuda:0")


def timeit(f, it=20):
    best = float("inf")
    for _ in range(3):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / it)
    return best


def worst(got, ref):
    ref = ref.float()
    bound = 8e-2 * ref.pow(2).mean().sqrt() + 3e-2 * ref.abs()
    return float(((got.float() - ref).abs() / bound).max())


def reference(q, k, v, do, hd, causal):
    qf = q[..., :hd].float().requires_grad_(True)
    kf = k[..., :hd].float().requires_grad_(True)
    vf = v[..., :hd].float().requires_grad_(True)
    rep = q.shape[1] // k.shape[1]
    s = qf @ kf.repeat_interleave(rep, 1).transpose(-1, -2) / math.sqrt(hd)
    if causal:
        S = q.shape[2]
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=dev), 1), float("-inf"))
    o = torch.softmax(s, -1) @ vf.repeat_interleave(rep, 1)
    o.permute(0, 2, 1, 3).backward(do.float())
    return qf.grad, kf.grad, vf.grad


def main():
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import _native as NV
    print(json.dumps(dict(library=str(NV.LIB_PATH))), flush=True)
    for name, B, H, HKV, S, hd, hdp, causal in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        pad = lambda t: torch.nn.functional.pad(t, (0, hdp - hd)).bfloat16().contiguous()
        q = pad(torch.randn(B, H, S, hd, device=dev, generator=g))
        k = pad(torch.randn(B, HKV, S, hd, device=dev, generator=g))
        v = pad(torch.randn(B, HKV, S, hd, device=dev, generator=g))
        o, lse = ops.attn_fwd(q, k, v, hd, causal)
        do = torch.randn(B, S, H, hd, device=dev, generator=g).bfloat16()
        rq, rk, rv = reference(q, k, v, do, hd, causal)
        frac = 0.5 if causal else 1.0
        flops = 10.0 * B * H * S * S * hd * frac   # five products
        row = dict(name=name)
        outs = []
        arms = (("r06_16x16", "2"), ("product", "0"), ("v32_both", "32")) + (("dq32_alt_build", "3"),)
        if os.environ.get("AB_DIAG"):   # timing diagnostics of dq32 (wrong results): no staging / no tile wait
            arms += (("diag_nostage", "5"), ("diag_nowait", "6"), ("diag_compute", "7"), ("diag_compute_edge", "8"))
        for arm, var in arms:
            os.environ["KD_ATTN_BWD_V"] = var
            dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, hd, causal)
            outs.append([t.clone() for t in (dq, dk, dv)])
            err = max(worst(dq[..., :hd], rq), worst(dk[..., :hd], rk), worst(dv[..., :hd], rv))
            ms = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, hd, causal))
            row[arm] = dict(us=round(ms * 1e3, 1), tflops=round(flops / ms / 1e9, 1), err_vs_bound=round(err, 3))
        os.environ.pop("KD_ATTN_BWD_V", None)
        row["arms_max_abs_diff"] = max(float((a[..., :hd].float() - b[..., :hd].float()).abs().max())
                                       for a, b in zip(outs[0], outs[1]))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
