import sys, torch
sys.path.insert(0, '/root/repo')
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops
dev = torch.device('cuda:0')
def deq(q, s): return q.view(torch.float8_e4m3fn).float() * s[:, None]
for (M, N, K) in [(300, 520, 160), (256, 256, 160), (300, 256, 64), (256, 520, 64), (256, 256, 128), (256,256,192)]:
    g = torch.Generator(device=dev).manual_seed(M * 7 + N)
    a = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=dev) * 0.05).to(torch.bfloat16)
    qa, sa = ops.quant_rows_fp8(a); qb, sb = ops.quant_rows_fp8(w)
    out = ops.gemm_fp8(qa, sa, qb, sb).float()
    ref = deq(qa, sa) @ deq(qb, sb).t()
    err = (out - ref).abs(); bad = err > (2**-7 * ref.abs() + 1e-3)
    r, c = bad.nonzero(as_tuple=True)
    print((M,N,K), "bad", int(bad.sum()), "rows", sorted(set((r//32).tolist()))[:20], "cols", sorted(set((c//32).tolist()))[:20], "max", float(err.max()))
    if bad.any():
        print("  rows mod 32", sorted(set((r % 32).tolist()))[:40])
        print("  cols mod 32", sorted(set((c % 32).tolist()))[:40])
