"""In-kernel stamps of the v8 GEMM (variant 17): where each wave's cycles go.
    python tools/stamp_gemm.py [M N K] [layout nt|nn|tn]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (6144, 37888, 3584)
lay = sys.argv[4] if len(sys.argv) > 4 else "nt"
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
if lay == "nt":
    a = torch.randn(M, K, device=dev, generator=g).bfloat16(); b = torch.randn(N, K, device=dev, generator=g).bfloat16()
elif lay == "nn":
    a = torch.randn(M, K, device=dev, generator=g).bfloat16(); b = torch.randn(K, N, device=dev, generator=g).bfloat16().t()
else:
    a = torch.randn(K, M, device=dev, generator=g).bfloat16().t(); b = torch.randn(K, N, device=dev, generator=g).bfloat16().t()
aux = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
ref = ops.gemm(a, b, variant=16, split_k=1)
for _ in range(3):
    out = ops.gemm(a, b, aux=aux, variant=17, split_k=1)
torch.cuda.synchronize()
assert torch.equal(out, ref), "stamp build changed the result"
blocks = ((M + 255) // 256) * ((N + 255) // 256)
st = aux.view(-1).view(torch.int32)[: blocks * 4 * 8].view(blocks * 4, 8).cpu().double()
names = ["prologue", "epi: LDS", "epi: store", "step sync", "units", "epilogue", "total"]
tot = st[:, 6].mean().item()
print(f"{M}x{N}x{K} {lay}: {blocks} blocks, {int(st[0, 7].item())} k-steps; mean cycles per wave")
for i, n in enumerate(names):
    col = st[:, i]
    print(f"  {n:10s} mean {col.mean().item():12.0f}  ({100 * col.mean().item() / tot:5.1f}%)  p10 {col.quantile(0.1).item():10.0f}  p90 {col.quantile(0.9).item():10.0f}")
print(f"  units per k-step {st[:, 4].mean().item() / st[0, 7].item():.0f} cycles (64 MFMA x 16 = 1024 ideal)")
