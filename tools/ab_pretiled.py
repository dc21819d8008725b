"""A/B of the pre-tiled B operand (kd_gemm_pretile) against the v8 kernel on the plain weights
(variant 24), on the teacher's forward GEMMs, in two cache states: warm (back-to-back calls) and
the step's (weights cold -- a 1 GiB write before each call -- and activations just written).
    python tools/ab_pretiled.py [--iters 12]"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SHAPES = [("t.gate_up+swiglu", 6144, 37888, 3584, "swiglu"), ("t.qkv", 6144, 4608, 3584, "qkv"),
          ("t.o+res", 6144, 3584, 3584, "res"), ("t.down+res", 6144, 3584, 18944, "res"),
          ("t.lm_head", 6144, 152064, 3584, "plain"), ("vit.fc1+gelu", 5832, 4304, 1152, "gelu")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    for name, M, N, K, kind in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, K, generator=g, device=dev).bfloat16()
        w = (torch.randn(N, K, generator=g, device=dev) * K ** -0.5).bfloat16()
        wt = ops.pretile_b(w, glu=kind == "swiglu")
        if kind == "swiglu":
            out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
            mk = lambda kw: (lambda: ops.gemm(x, w, out=out, act="swiglu", **kw))
        elif kind == "qkv":
            S, nq, nkv, hd = 1536, 28, 4, 128
            bias = torch.randn(N, generator=g, device=dev).bfloat16()
            inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float32, device=dev) / hd))
            f = torch.arange(S, dtype=torch.float32, device=dev)[:, None] * inv[None]
            cos, sin = f.cos().contiguous(), f.sin().contiguous()
            q = torch.empty((M // S, nq, S, hd), dtype=torch.bfloat16, device=dev)
            k = torch.empty((M // S, nkv, S, hd), dtype=torch.bfloat16, device=dev)
            v = torch.empty((M // S, nkv, S, hd), dtype=torch.bfloat16, device=dev)
            mk = lambda kw: (lambda: ops.gemm_qkv(x, w, bias, q, k, v, S, nq, nkv, hd, hd, cos, sin, **kw))
        elif kind == "res":
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            res = torch.randn(M, N, generator=g, device=dev).bfloat16()
            mk = lambda kw: (lambda: ops.gemm(x, w, out=out, residual=res, split_k=1, **kw))
        elif kind == "gelu":
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            bias = torch.randn(N, generator=g, device=dev).bfloat16()
            mk = lambda kw: (lambda: ops.gemm(x, w, out=out, bias=bias, act="gelu_tanh", split_k=1, **kw))
        else:
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            mk = lambda kw: (lambda: ops.gemm(x, w, out=out, split_k=1, **kw))
        fns = {"v8": mk(dict(variant=24)), "pretiled": mk(dict(b_pretiled=wt))}
        res_t = {}
        for r in range(2):
            for key, fn in (fns.items() if r == 0 else list(fns.items())[::-1]):
                fn()
                torch.cuda.synchronize()
                # warm: back to back
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res_t.setdefault(f"{key}_warm_us", []).append(e0.elapsed_time(e1) / a.iters * 1e3)
                ts = []
                for _ in range(a.iters):
                    junk.fill_(1.0)
                    x.mul_(1.0)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                ts.sort()
                res_t.setdefault(f"{key}_cold_us", []).append(ts[len(ts) // 2])
        print(name, f"M={M} N={N} K={K}", json.dumps({k_: round(min(v_), 1) for k_, v_ in res_t.items()}), flush=True)


if __name__ == "__main__":
    main()
