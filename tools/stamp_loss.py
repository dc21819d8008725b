"""Where k_loss_grad_loca_rr's time goes: per-workgroup s_memtime cycles per phase of a row (the A/B
library with KD_RR_STAMPS=1; wave 0 of each workgroup), at the c1 shape (LoCa T = 1, random logits).
    KDSTEP_LIB=tools/ab/libkdstep_ab.so KD_RR_STAMPS=1 python tools/stamp_loss.py"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import _native as NV, ops  # noqa: E402

B, L, Vs, Vt = 4, 1536, 151936, 152064
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
s = (torch.randn(B, L, Vs, device=dev, generator=g) * 2).bfloat16()
t = (torch.randn(B, L, Vt, device=dev, generator=g) * 2).bfloat16()
lab = torch.randint(0, 151643, (B, L), device=dev, generator=g)
lib = NV.lib()
f = lib.kd_ab_rr_stamps
f.argtypes = [C.c_void_p, C.c_int, C.c_int]
ops.kd_loss_fwd_bwd(s, t, lab, "loca", temperature=1.0)
f(None, 0, 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
ops.kd_loss_fwd_bwd(s, t, lab, "loca", temperature=1.0)
e1.record()
torch.cuda.synchronize()
buf = np.zeros(4096 * 8, dtype=np.uint64)
f(buf.ctypes.data, buf.size, 0)
st = buf.reshape(4096, 8)
used = st[:, 4] > 0
st = st[used].astype(np.float64)
rows = st[:, 4]
names = ["loads + pass A", "block sums", "hand-off", "pass B + stores"]
tot = st[:, :4].sum(1)
print(f"workgroups {used.sum()}, rows per workgroup {rows.mean():.1f}, whole loss {e0.elapsed_time(e1) * 1e3:.0f} us")
for k, n in enumerate(names):
    per = st[:, k] / rows
    print(f"  {n:16s} mean {per.mean():8.0f} cycles/row  ({st[:, k].sum() / tot.sum() * 100:5.1f} %)  p10 {np.percentile(per, 10):8.0f}  p90 {np.percentile(per, 90):8.0f}")
print(f"  total            mean {(tot / rows).mean():8.0f} cycles/row")
