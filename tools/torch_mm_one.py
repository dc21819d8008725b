"""torch.mm (hipBLASLt) on one GEMM shape, for PMC comparison with kd_gemm.
    python tools/torch_mm_one.py M N K [iters]"""
import sys

import torch

M, N, K = (int(x) for x in sys.argv[1:4])
it = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
a = torch.randn(M, K, device=dev, generator=g).bfloat16()
b = torch.randn(N, K, device=dev, generator=g).bfloat16()
for _ in range(it):
    c = a @ b.t()
torch.cuda.synchronize()
