"""In-kernel stamps of the fused gate|up + SwiGLU GEMM (k_gemm8 SwiGLU build, forced variant 28):
per wave, cycles in the prologue, the k-loop, the step-end syncs and the epilogue's three phases
(bf16 staging of the accumulators in LDS, the aux pre-activation pass, the silu(gate) * up pass).
    python tools/stamp_glu.py [M N K] [--aux]     (N = 2I; default the teacher 6144 37888 3584)"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
M, N, K = (int(x) for x in args[:3]) if len(args) >= 3 else (6144, 37888, 3584)
want_aux = "--aux" in sys.argv
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
a = torch.randn(M, K, device=dev, generator=g).bfloat16()
b = torch.randn(N, K, device=dev, generator=g).bfloat16()
aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if want_aux else None
aux_ref = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if want_aux else None
ref = ops.gemm(a, b, act="swiglu", aux=aux_ref, variant=16, split_k=1)
blocks = ((M + 255) // 256) * (N // 256)
for _ in range(3):
    out = ops.gemm(a, b, act="swiglu", aux=aux, variant=28)
torch.cuda.synchronize()
assert torch.equal(out, ref), "stamp build changed the result"
if want_aux:
    assert torch.equal(aux, aux_ref), "stamp build changed the aux output"
ws = ops._workspace(("gemm_splitk", ops._stream()), ops.GEMM_SPLITK_WS, dev)
st = ws[: blocks * 4 * 8 * 4].view(torch.int32).view(blocks * 4, 8).cpu().double()
tot = st[:, 6].mean().item()
epi = st[:, 5]
rows = [("prologue", st[:, 0]), ("k-loop units", st[:, 4]), ("step sync", st[:, 3]),
        ("epi: LDS staging", st[:, 1]), ("epi: aux pass", st[:, 2]), ("epi: silu*up pass", epi - st[:, 1] - st[:, 2]),
        ("epilogue total", epi), ("total", st[:, 6])]
print(f"{M}x{N}x{K} swiglu{' +aux' if want_aux else ''}: {blocks} tiles, {int(st[0, 7].item())} k-steps; mean cycles per wave")
for n, col in rows:
    print(f"  {n:18s} mean {col.mean().item():10.0f}  ({100 * col.mean().item() / tot:5.1f}%)  p10 {col.quantile(0.1).item():9.0f}"
          f"  p90 {col.quantile(0.9).item():9.0f}")
