"""Isolated timing of the norm backward (k_norm_bwd + k_reduce_parts) and forward on the
step's shapes (run under rocprofv3 --kernel-trace --stats for per-kernel times).
    python tools/bench_norm.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for R, D, rms in ((6144, 896, True), (5832, 1152, False)):   # the backward shapes (D <= 2048)
    x = torch.randn(R, D, device=dev, generator=g).bfloat16()
    w = torch.randn(D, device=dev, generator=g).bfloat16()
    b = torch.randn(D, device=dev, generator=g).bfloat16()
    dy = torch.randn(R, D, device=dev, generator=g).bfloat16()
    y, mean, rstd = ops.norm_fwd(x, w, None if rms else b, 1e-6, rms=rms, save_stats=True)
    dx = torch.zeros(R, D, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(D, device=dev)
    db = None if rms else torch.zeros(D, device=dev)
    for _ in range(20):
        ops.norm_bwd(x, w, dy, mean, rstd, dx=dx, dx_accum=True, dweight=dw, dbias=db, rms=rms)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.norm_bwd(x, w, dy, mean, rstd, dx=dx, dx_accum=True, dweight=dw, dbias=db, rms=rms)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    gb = R * D * 2 * 4 / 1e9   # x, dy, dx read, dx write
    print(f"norm_bwd R={R} D={D} rms={rms}: {ms * 1e3:.1f} us/call ({gb / ms * 1e3 / 1e3:.2f} TB/s incl. reduce)", flush=True)
