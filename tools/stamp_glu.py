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

# per-CU placement (wave 0 of each workgroup): start / end on the 100 MHz real-time clock, HW_ID, XCC_ID;
# the gap between one workgroup's end and the next one's start on the same CU is time no stamp above sees
pl = ws[blocks * 4 * 8 * 4: blocks * (4 * 8 + 4) * 4].view(torch.int32).view(blocks, 4).cpu().numpy().astype("int64")
import collections
import numpy as np
start, end = pl[:, 0] & 0xFFFFFFFF, pl[:, 1] & 0xFFFFFFFF
hw, xcc = pl[:, 2], pl[:, 3] & 0xF
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
key = xcc * 1000 + se * 100 + cu
per = collections.defaultdict(list)
for k, s0, e0 in zip(key, start, end):
    per[k].append((s0, e0))
gaps, lens, counts = [], [], []
for k, v in per.items():
    v.sort()
    counts.append(len(v))
    lens += [e - s for s, e in v]
    gaps += [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
t0, t1 = start.min(), end.max()
g = np.array(gaps) * 10.0   # ns
ln = np.array(lens) * 10.0
print(f"  placement: {len(per)} CUs used, workgroups per CU min {min(counts)} max {max(counts)}; launch span {(t1 - t0) / 100:.1f} us")
print(f"  workgroup life mean {ln.mean() / 1e3:.2f} us; gap to the CU's next workgroup mean {g.mean() / 1e3:.2f} us "
      f"p10 {np.quantile(g, 0.1) / 1e3:.2f} p90 {np.quantile(g, 0.9) / 1e3:.2f}  ({100 * g.sum() / (g.sum() + ln.sum()):.1f}% of CU time)")
print(f"  in-kernel clock: {st[:, 6].mean().item() / (ln.mean() / 1e3):.0f} MHz (mean wave cycles / mean workgroup life)")
