"""How many launches can the host queue on one stream behind a long-running kernel before
hipLaunchKernel blocks (the runtime's in-flight limit), for a small-kernarg torch kernel
and for kd_gemm (432-B kernarg):
    python tools/launch_depth.py"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402


def probe(name, launch, n=6000, streams=1):
    ss = [torch.cuda.Stream() for _ in range(streams)]
    for s in ss:
        with torch.cuda.stream(s):
            torch.cuda._sleep(4_000_000_000)      # ~1-2 s of spinning on each stream
    t = []
    for i in range(n):
        s = ss[i % streams]
        with torch.cuda.stream(s):
            t0 = time.perf_counter()
            launch()
            t.append(time.perf_counter() - t0)
    first_block = next((i for i, x in enumerate(t) if x > 5e-3), None)
    torch.cuda.synchronize()
    print(f"{name} streams={streams}: first launch > 5 ms at index {first_block}; "
          f"median {1e6 * sorted(t)[len(t) // 2]:.1f} us", flush=True)


x = torch.zeros(16, device="cuda")
a = torch.randn(64, 64, device="cuda").bfloat16()
b = torch.randn(64, 64, device="cuda").bfloat16()
c = torch.empty(64, 64, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
probe("torch add_ (small kernarg)", lambda: x.add_(1))
probe("kd_gemm 64^3 (432-B kernarg)", lambda: ops.gemm(a, b, out=c))
probe("kd_gemm 64^3, 2 streams", lambda: ops.gemm(a, b, out=c), streams=2)
ev = torch.cuda.Event()
probe("event record + add_", lambda: (ev.record(), x.add_(1)))
