"""A/B of the SwiGLU GEMM epilogue (packed rewrite vs KD_GLU_EPI_V0=1, the previous one) on the
step's two gate|up shapes: warm back-to-back calls and calls with the weights evicted (cold).
    python tools/ab_glu_epi.py [--iters 10]"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

iters = int(sys.argv[sys.argv.index("--iters") + 1]) if "--iters" in sys.argv else 10
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)
shapes = [("teacher", 6144, 37888, 3584, False), ("student", 6144, 9728, 896, True)]


def timed(f, cold):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        if cold:
            junk.fill_(1.0)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for name, M, N, K, want_aux in shapes:
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    b = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if want_aux else None
    outs = {}
    res = {}
    for rep in range(2):
        for v0 in ("0", "1"):
            os.environ["KD_GLU_EPI_V0"] = v0
            f = lambda: ops.gemm(a, b, act="swiglu", aux=aux)
            outs[v0] = f().clone()
            for cold in (False, True):
                res.setdefault((v0, cold), []).append(timed(f, cold))
    os.environ["KD_GLU_EPI_V0"] = "0"
    assert torch.equal(outs["0"], outs["1"]), "epilogues disagree"
    fl = 2.0 * M * N * K
    for cold in (False, True):
        new, old = min(res[("0", cold)]), min(res[("1", cold)])
        print(f"{name} {M}x{N}x{K}{' +aux' if want_aux else ''} {'cold' if cold else 'warm'}: packed {new:8.1f} us "
              f"({fl / new / 1e6:6.0f} TF/s)  previous {old:8.1f} us ({fl / old / 1e6:6.0f} TF/s)  {100 * (new / old - 1):+.1f}%")
