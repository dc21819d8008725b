"""Pre-tiled B (kd_gemm_pretile + kd_gemm_desc.b_pretiled): the weights rewritten once as the
256x256 kernel's per-tile stage images, so every LDS-DMA reads one contiguous KiB.  The LDS image is
the same, so the GEMM is bit-identical to the v8 kernel on the plain [N, K] weights (variant 24,
unsplit): plain and every epilogue, the fused SwiGLU (gate|up row gather baked into the tiles), the
q|k|v scatter, partial tiles in M and N and K tails of every length."""
import pytest
import torch

from test_gemm_gpu import _check, _ops, _rand

pytestmark = pytest.mark.gpu

# M*N >= 2^20: the shapes variant 24 runs on the 256x256 v8 kernel (smaller ones take the 128x128
# kernel, whose epilogue rounds differently)
SHAPES = [(1024, 1024, 32), (1024, 1024, 40), (1300, 1032, 4304), (1040, 1048, 600), (1029, 1040, 72),
          (2048, 768, 96), (1024, 1024, 2248), (1024, 1024, 8), (1536, 4608, 3584)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_pretiled_bitexact_vs_v8(M, N, K, dev):
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=401)
    w = _rand(N, K, dev=dev, seed=402, scale=0.05)
    wt = ops.pretile_b(w)
    o = ops.gemm(a, w, b_pretiled=wt, split_k=1)
    assert torch.equal(o, ops.gemm(a, w, variant=24, split_k=1))
    _check(o, a.float() @ w.float().t())
    bias = _rand(N, dev=dev, seed=403)
    res = _rand(M, N, dev=dev, seed=404)
    ax = [torch.empty(M, N, dtype=torch.bfloat16, device=dev) for _ in range(2)]
    r = [ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=res, aux=ax[0], b_pretiled=wt, split_k=1),
         ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=res, aux=ax[1], variant=24, split_k=1)]
    assert torch.equal(r[0], r[1]) and torch.equal(ax[0], ax[1])
    g = torch.Generator(device=dev).manual_seed(405)
    r32 = torch.randn(M, N, generator=g, device=dev)
    f = [ops.gemm(a, w, bias=bias, residual=r32, out_dtype=torch.float32, b_pretiled=wt, split_k=1),
         ops.gemm(a, w, bias=bias, residual=r32, out_dtype=torch.float32, variant=24, split_k=1)]
    assert torch.equal(f[0], f[1])
    if N % 256 == 0:
        wg = ops.pretile_b(w, glu=True)
        gu = [torch.empty(M, N, dtype=torch.bfloat16, device=dev) for _ in range(2)]
        sw = [ops.gemm(a, w, act="swiglu", aux=gu[0], b_pretiled=wg), ops.gemm(a, w, act="swiglu", aux=gu[1], variant=24)]
        assert torch.equal(sw[0], sw[1]) and torch.equal(gu[0], gu[1])


def test_pretiled_qkv_scatter_teacher(dev):
    ops = _ops()
    B, S, K, nq, nkv, hd, hdp = 1, 1536, 3584, 28, 4, 128, 128
    M, N = B * S, (nq + 2 * nkv) * hd
    x = _rand(M, K, dev=dev, seed=420)
    w = _rand(N, K, dev=dev, seed=421, scale=0.05)
    bias = _rand(N, dev=dev, seed=422)
    inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
    f = torch.arange(S, dtype=torch.float32)[:, None] * inv[None]
    cos, sin = f.cos().to(dev).contiguous(), f.sin().to(dev).contiguous()
    wt = ops.pretile_b(w)
    outs = []
    for kw in (dict(b_pretiled=wt), dict(variant=24)):
        q = torch.empty((B, nq, S, hdp), dtype=torch.bfloat16, device=dev)
        k = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
        v = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
        ops.gemm_qkv(x, w, bias, q, k, v, S, nq, nkv, hd, hdp, cos, sin, **kw)
        outs.append((q, k, v))
    torch.cuda.synchronize()
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)


def test_pretiled_rejects_split(dev):
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import _native as NV
    ops = _ops()
    a = _rand(512, 4096, dev=dev, seed=430)
    w = _rand(512, 4096, dev=dev, seed=431)
    with pytest.raises(NV.KdError):
        ops.gemm(a, w, b_pretiled=ops.pretile_b(w), split_k=2)
