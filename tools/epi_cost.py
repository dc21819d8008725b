"""Epilogue cost of the fused GEMM builds on the step's shapes, warm (back-to-back) and cold
(a 1 GiB write between calls evicts the Infinity Cache and the L2s), HIP events:
  q|k|v scatter (+RoPE) vs the plain bias GEMM; fp32-residual o_proj vs plain; dgrad with the
  dSwiGLU / dGELU epilogue (aux read, [M, 2I] write) vs the plain dgrad.
    python tools/epi_cost.py [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)


def rnd(*s, sc=1.0):
    return (torch.randn(*s, device=dev, generator=g) * sc).bfloat16()


def timed(f, cold):
    ts = []
    for i in range(it + 1):
        if cold:
            junk.fill_(float(i))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def row(name, fs):
    out = []
    for label, f in fs:
        out.append(f"{label} warm {timed(f, False):7.1f} cold {timed(f, True):7.1f}")
    print(f"{name:34s} " + " | ".join(out), flush=True)


# q|k|v: teacher (S 1536, 28 q / 4 kv heads of 128) and SigLIP (S 729, 16 heads of 72 -> 96)
for name, B, S, nq, nkv, hd, hdp, K, rope in (("t.qkv 6144x4608x3584", 4, 1536, 28, 4, 128, 128, 3584, True),
                                              ("vit.qkv 5832x3456x1152", 8, 729, 16, 16, 72, 96, 1152, False)):
    M, N = B * S, (nq + 2 * nkv) * hd
    x, w, bias = rnd(M, K), rnd(N, K, sc=0.05), rnd(N)
    q = torch.empty(B, nq, S, hdp, dtype=torch.bfloat16, device=dev)
    k = torch.empty(B, nkv, S, hdp, dtype=torch.bfloat16, device=dev)
    v = torch.empty(B, nkv, S, hdp, dtype=torch.bfloat16, device=dev)
    cos = torch.rand(S, hd // 2, device=dev) if rope else None
    sin = torch.rand(S, hd // 2, device=dev) if rope else None
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    row(name, [("plain", lambda: ops.gemm(x, w, out, bias=bias)),
               ("scatter", lambda: ops.gemm_qkv(x, w, bias, q, k, v, S, nq, nkv, hd, hdp, cos, sin))])

# o_proj / down_proj with the fp32 residual stream
for name, M, N, K in (("t.o 6144x3584x3584", 6144, 3584, 3584), ("s.down 6144x896x4864", 6144, 896, 4864),
                      ("vit.fc2 5832x1152x4304", 5832, 1152, 4304)):
    x, w = rnd(M, K), rnd(N, K, sc=0.05)
    r32 = torch.randn(M, N, device=dev, generator=g)
    o16 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    o32 = torch.empty(M, N, dtype=torch.float32, device=dev)
    row(name, [("plain", lambda: ops.gemm(x, w, o16)),
               ("f32 resid", lambda: ops.gemm(x, w, o32, residual=r32, out_dtype=torch.float32))])

# dgrad + activation backward: dY [M, H] . W [H, I] (W stored [H, I] row-major = MN-major B)
for name, M, I, H, act in (("s.down dgrad+dswiglu 6144x4864x896", 6144, 4864, 896, "dswiglu"),
                           ("vit.fc2 dgrad+dgelu 5832x4304x1152", 5832, 4304, 1152, "dgelu_tanh")):
    dy, w = rnd(M, H), rnd(H, I, sc=0.05)
    aux = rnd(M, 2 * I if act == "dswiglu" else I)
    o = torch.empty(M, I, dtype=torch.bfloat16, device=dev)
    od = torch.empty(M, 2 * I if act == "dswiglu" else I, dtype=torch.bfloat16, device=dev)
    row(name, [("plain", lambda: ops.gemm(dy, w.t(), o, split_k=1)),
               ("dact", lambda: ops.gemm(dy, w.t(), od, act=act, aux=aux, split_k=1))])
