"""Time the fused KD loss (kd_loss_fwd_bwd) at the c1 shape and report its HBM roofline.
    python tools/bench_loss.py [B] [variant]
Algorithmic bytes: read teacher + student logits, write dlogits = 3 x B*L*V_s x 2 B."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
var = sys.argv[2] if len(sys.argv) > 2 else "loca"
L, Vs, Vt = 1536, 151936, 152064
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
s = (torch.randn(B, L, Vs, device=dev, generator=g) * 2).bfloat16()
t = (torch.randn(B, L, Vt, device=dev, generator=g) * 2).bfloat16()
# bench-like labels (labels = input ids: 24 + 27 random text ids around 1485 image tokens)
lab = torch.full((B, L), 151646, dtype=torch.int64, device=dev)
lab[:, :24] = torch.randint(0, 151643, (B, 24), device=dev, generator=g)
lab[:, -27:] = torch.randint(0, 151643, (B, 27), device=dev, generator=g)
f = lambda: ops.kd_loss_fwd_bwd(s, t, lab, var, temperature=1.0)
f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e30
for _ in range(3):
    e0.record()
    for _ in range(5):
        f()
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) / 5)
alg = 3.0 * B * L * Vs * 2
print(f"kd_loss {var} B={B}: {best * 1e3:.0f} us  algorithmic {alg / 1e9:.2f} GB -> {alg / best / 1e6:.0f} GB/s "
      f"({alg / best / 1e6 / 8000:.2f} of 8 TB/s)")
