"""Forward GEMMs of the KD step timed the way the step runs them: the weights COLD (a 1 GiB write
between calls evicts the 256 MB Infinity Cache and the L2s: every teacher / student layer reads
weights it last touched a whole step ago) and the activation operand WARM (re-written just before
the call, as the producing kernel would).  One call per timing, HIP events around it, median over
--iters calls; builds compared: auto plan (0), v8 (24), v12 (26) and the v3 tiles (5/6/7).
    python tools/ab_cold.py [--iters 12] [--variants 0,24,26] [--only name]"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

SHAPES = [  # name, M, N, K, kind
    ("t.qkv", 6144, 4608, 3584, "qkv:4,1536,28,4,128,128,1"),
    ("t.o+res", 6144, 3584, 3584, "res"),
    ("t.gate_up+swiglu", 6144, 37888, 3584, "swiglu"),
    ("t.down+res", 6144, 3584, 18944, "res"),
    ("t.lm_head", 6144, 152064, 3584, "plain"),
    ("s.qkv", 6144, 1152, 896, "qkv:4,1536,14,2,64,64,1"),
    ("s.o+res32", 6144, 896, 896, "res32"),
    ("s.gate_up+swiglu", 6144, 9728, 896, "swiglu_aux"),
    ("s.down+res32", 6144, 896, 4864, "res32"),
    ("vit.qkv", 5832, 3456, 1152, "qkv:8,729,16,16,72,96,0"),
    ("vit.o+res32", 5832, 1152, 1152, "res32"),
    ("vit.fc1+gelu", 5832, 4304, 1152, "gelu"),
    ("vit.fc2+res32", 5832, 1152, 4304, "res32"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--variants", default="0,24,26")
    ap.add_argument("--only", default=None)
    ap.add_argument("--prefetch", action="store_true",
                    help="also time kd_prefetch(weights) + the GEMM together (the plan's build), residual re-written too")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    vs = [int(v) for v in a.variants.split(",")]
    junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    for name, M, N, K, kind in SHAPES:
        if a.only and a.only not in name:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, K, generator=g, device=dev).bfloat16()
        w = (torch.randn(N, K, generator=g, device=dev) * K ** -0.5).bfloat16()
        extra = {}
        res = None
        if kind.startswith("qkv"):
            B, S, nq, nkv, hd, hdp, rope = (int(t) for t in kind.split(":")[1].split(","))
            bias = torch.randn(N, generator=g, device=dev).bfloat16()
            cos = sin = None
            if rope:
                inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float32, device=dev) / hd))
                f = torch.arange(S, dtype=torch.float32, device=dev)[:, None] * inv[None]
                cos, sin = f.cos().contiguous(), f.sin().contiguous()
            q = torch.empty((B, nq, S, hdp), dtype=torch.bfloat16, device=dev)
            k = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
            v = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
            call = lambda var: ops.gemm_qkv(x, w, bias, q, k, v, S, nq, nkv, hd, hdp, cos, sin, variant=var)
        elif kind in ("swiglu", "swiglu_aux"):
            out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if kind == "swiglu_aux" else None
            call = lambda var: ops.gemm(x, w, out=out, act="swiglu", aux=aux, variant=var)
        elif kind == "gelu":
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            bias = torch.randn(N, generator=g, device=dev).bfloat16()
            call = lambda var: ops.gemm(x, w, out=out, bias=bias, act="gelu_tanh", aux=aux, variant=var)
        elif kind == "res":
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            res = torch.randn(M, N, generator=g, device=dev).bfloat16()
            call = lambda var: ops.gemm(x, w, out=out, residual=res, variant=var)
        elif kind == "res32":
            out = torch.empty(M, N, dtype=torch.float32, device=dev)
            res = torch.randn(M, N, generator=g, device=dev)
            bias = torch.randn(N, generator=g, device=dev).bfloat16()
            call = lambda var: ops.gemm(x, w, out=out, bias=bias, residual=res, out_dtype=torch.float32, variant=var)
        else:
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            call = lambda var: ops.gemm(x, w, out=out, variant=var)
        res_t = {}
        warm_extra = [res] if isinstance(res, torch.Tensor) else []
        if a.prefetch:
            from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import _native as NV
            for mode in ("cold", "prefetch"):
                ts = []
                for i in range(a.iters):
                    junk.fill_(1.0)
                    x.mul_(1.0)
                    for t_ in warm_extra:
                        t_.mul_(1.0)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    if mode == "prefetch":
                        NV.call("kd_prefetch", w.data_ptr(), w.numel() * 2, 0, ops._stream())
                    call(0)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                ts.sort()
                res_t[f"{mode}_us"] = round(ts[len(ts) // 2], 1)
            print(name, f"M={M} N={N} K={K} W={w.numel() * 2 / 1e6:.1f}MB", json.dumps(res_t), flush=True)
            continue
        for var in vs:
            try:
                call(var)
            except Exception as e:   # a build that does not take this epilogue
                res_t[f"v{var}"] = repr(e)[:60]
                continue
            ts = []
            for i in range(a.iters):
                junk.fill_(1.0)          # evict the Infinity Cache and the L2s (weights cold)
                x.mul_(1.0)              # the activation operand just written (warm), as in the step
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                call(var)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            res_t[f"v{var}_us"] = round(ts[len(ts) // 2], 1)
        print(name, f"M={M} N={N} K={K}", json.dumps(res_t), flush=True)


if __name__ == "__main__":
    main()
