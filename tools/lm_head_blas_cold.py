"""The lm_head GEMMs of the c1 step (teacher 6144 x 152064 x 3584, student 6144 x 151936 x 896; C = A B^T,
bf16 out) in the step's cache state (the weight read once per step: a 1 GiB write before each call evicts
the L2s and the Infinity Cache; the activation just written): kd_gemm vs torch.mm (hipBLASLt), interleaved.
    python tools/lm_head_blas_cold.py [iters]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)
for M, N, K in ((6144, 152064, 3584), (6144, 151936, 896), (6144, 4608, 3584), (6144, 3584, 3584)):
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    res = {"kd": [], "blas": []}
    fns = {"kd": lambda: ops.gemm(a, w, out=out), "blas": lambda: torch.mm(a, w.t(), out=out)}
    for f in fns.values():
        f()
    for _ in range(it):
        for k, f in fns.items():
            junk.fill_(1.0)
            a.mul_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print(f"{M}x{N}x{K} cold: kd {med['kd']:.1f} us ({fl / med['kd'] / 1e6:.0f} TF/s)  hipblaslt {med['blas']:.1f} us "
          f"({fl / med['blas'] / 1e6:.0f} TF/s)", flush=True)
