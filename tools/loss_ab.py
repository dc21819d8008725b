"""A/B of the fused KD loss between two builds of the library: time of kd_loss_fwd_bwd at the c1 shape
(LoCa, T = 1, random logits, bench-like labels) and a digest of its outputs (the four loss terms and
every dlogits bit), so a rewritten kernel can be shown bit-identical to the previous build.
    KDSTEP_LIB=<lib.so> python tools/loss_ab.py [B] [iters]"""
import hashlib
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
L, Vs, Vt = 1536, 151936, 152064
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
s = (torch.randn(B, L, Vs, device=dev, generator=g) * 2).bfloat16()
t = (torch.randn(B, L, Vt, device=dev, generator=g) * 2).bfloat16()
lab = torch.full((B, L), 151646, dtype=torch.int64, device=dev)
lab[:, :24] = torch.randint(0, 151643, (B, 24), device=dev, generator=g)
lab[:, -27:] = torch.randint(0, 151643, (B, 27), device=dev, generator=g)
loss = torch.empty(4, dtype=torch.float32, device=dev)
d = torch.empty((B, L, Vs), dtype=torch.bfloat16, device=dev)
f = lambda: ops.kd_loss_fwd_bwd(s, t, lab, "loca", temperature=1.0, want_grad=True, loss_out=loss, dlogits_out=d)
f()
torch.cuda.synchronize()
h = hashlib.sha256(d.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
terms = [float(x) for x in loss.cpu()]
ts = []
for _ in range(iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    f()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
ts.sort()
print(f"[{os.path.basename(os.environ.get('KDSTEP_LIB', 'libkdstep.so'))}] kd_loss loca B={B}: median {ts[len(ts) // 2]:.0f} us "
      f"min {ts[0]:.0f} us  terms {terms}  dlogits sha256 {h}")
