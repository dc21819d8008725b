import sys; sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import torch
from test_attention_gpu import _inputs, _ref
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops
dev = torch.device("cuda:0")
for (B, H, HKV, S, hd, hdp, causal) in [(2, 4, 2, 200, 64, 64, True), (1, 4, 2, 200, 64, 64, True), (2,4,2,192,64,64,True), (2,2,2,200,64,64,True), (2,4,2,256,64,64,True), (1,2,1,200,64,64,False)]:
    q, k, v = _inputs(B, H, HKV, S, hd, hdp, dev, seed=1)
    o, lse = ops.attn_fwd(q, k, v, hd, causal)
    g = torch.Generator().manual_seed(2)
    do = torch.randn(B, S, H, hd, generator=g).to(dev, torch.bfloat16)
    dq, dk, dv = ops.attn_bwd(q, k, v, o, do, lse, hd, causal)
    qf = q[..., :hd].float().requires_grad_(True); kf = k[..., :hd].float().requires_grad_(True); vf = v[..., :hd].float().requires_grad_(True)
    ro, _ = _ref(qf, kf, vf, causal, hd)
    ro.permute(0, 2, 1, 3).backward(do.float())
    for name, got, ref in (("dq", dq[..., :hd], qf.grad), ("dk", dk[..., :hd], kf.grad), ("dv", dv[..., :hd], vf.grad)):
        err = (got.float() - ref).abs()
        rel = err / (ref.pow(2).mean().sqrt())
        idx = torch.nonzero(rel == rel.max())[0].tolist()
        print((B,H,HKV,S,causal), name, "max rel-to-rms %.3e" % rel.max().item(), "at", idx, "got", got.float()[tuple(idx)].item(), "ref", ref[tuple(idx)].item())
