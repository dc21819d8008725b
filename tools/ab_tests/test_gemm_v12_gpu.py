"""v12 GEMM (v8's tiles, MFMAs and accumulation order with whole-cache-line staging of
K-major operands: stage pairs of 64 k, 8 rows x 128 B per DMA instruction; forced variant
26) is bit-identical to v8 (variant 24) on every K-major x K-major GEMM: plain, every
epilogue (bias, activations, row-modulus residual, aux, fp32 residual / output, accumulate,
alpha x device scalar), the fused SwiGLU and q|k|v scatter builds, split-K planes, partial
tiles and K tails of every length (incl. K shorter than the prefetch ring).  Forced variant 27 is
v12 without the barriers at the end of odd steps (the pair-granular hazards need only the even
ones, g12_tile): bit-identical too."""
import pytest
import torch

from test_gemm_gpu import _check, _ops, _rand

pytestmark = pytest.mark.gpu

SHAPES = [(256, 256, 32), (256, 256, 40), (512, 512, 256), (1458, 1152, 1152), (1000, 904, 600), (300, 272, 4304),
          (257, 520, 72), (6144 // 4, 4608, 3584 // 4), (128, 384, 4864), (512, 768, 96), (512, 768, 160),
          (384, 512, 2248), (256, 256, 8)]


@pytest.mark.parametrize("v12", [26, 27])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_v12_bitexact_vs_v8(M, N, K, v12, dev):
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=301)
    w = _rand(N, K, dev=dev, seed=302, scale=0.05)
    o12 = ops.gemm(a, w, variant=v12, split_k=1)
    assert torch.equal(o12, ops.gemm(a, w, variant=24, split_k=1))
    _check(o12, a.float() @ w.float().t())
    bias = _rand(N, dev=dev, seed=303)
    res = _rand(M, N, dev=dev, seed=304)
    ax = [torch.empty(M, N, dtype=torch.bfloat16, device=dev) for _ in range(2)]
    o = [ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=res, aux=ax[i], variant=v, split_k=1)
         for i, v in enumerate((v12, 24))]
    assert torch.equal(o[0], o[1]) and torch.equal(ax[0], ax[1])
    g = torch.Generator(device=dev).manual_seed(305)
    r32 = torch.randn(M, N, generator=g, device=dev)
    f = [ops.gemm(a, w, bias=bias, residual=r32, out_dtype=torch.float32, variant=v, split_k=1) for v in (v12, 24)]
    assert torch.equal(f[0], f[1])
    s = torch.tensor([2.0], device=dev)
    acc = [torch.full((M, N), 2.0, device=dev) for _ in range(2)]
    for i, v in enumerate((v12, 24)):
        ops.gemm(a, w, out=acc[i], accumulate=True, variant=v, alpha=0.25, alpha_dev=s)
    assert torch.equal(acc[0], acc[1])
    if N % 256 == 0:
        gu = [torch.empty(M, N, dtype=torch.bfloat16, device=dev) for _ in range(2)]
        sw = [ops.gemm(a, w, act="swiglu", aux=gu[i], variant=v) for i, v in enumerate((v12, 24))]
        assert torch.equal(sw[0], sw[1]) and torch.equal(gu[0], gu[1])


@pytest.mark.parametrize("v12", [26, 27])
@pytest.mark.parametrize("split", [2, 3])
def test_v12_split_k(split, v12, dev):
    ops = _ops()
    M, N, K = 520, 384, 4296
    a = _rand(M, K, dev=dev, seed=310)
    w = _rand(N, K, dev=dev, seed=311, scale=0.05)
    assert torch.equal(ops.gemm(a, w, variant=v12, split_k=split), ops.gemm(a, w, variant=24, split_k=split))


@pytest.mark.parametrize("v12", [26, 27])
@pytest.mark.parametrize("shape", ["teacher", "student", "siglip"])
def test_v12_qkv_scatter(shape, v12, dev):
    ops = _ops()
    B, S, K, nq, nkv, hd, hdp, rope = {
        "teacher": (1, 1536, 3584, 28, 4, 128, 128, True),
        "student": (2, 1536, 896, 14, 2, 64, 64, True),
        "siglip": (2, 729, 1152, 16, 16, 72, 96, False)}[shape]
    M, N = B * S, (nq + 2 * nkv) * hd
    x = _rand(M, K, dev=dev, seed=320)
    w = _rand(N, K, dev=dev, seed=321, scale=0.05)
    bias = _rand(N, dev=dev, seed=322)
    cos = sin = None
    if rope:
        inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
        f = torch.arange(S, dtype=torch.float32)[:, None] * inv[None]
        cos, sin = f.cos().to(dev).contiguous(), f.sin().to(dev).contiguous()
    outs = []
    for v in (v12, 24):
        q = torch.empty((B, nq, S, hdp), dtype=torch.bfloat16, device=dev)
        k = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
        vv = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
        ops.gemm_qkv(x, w, bias, q, k, vv, S, nq, nkv, hd, hdp, cos, sin, variant=v)
        outs.append((q, k, vv))
    torch.cuda.synchronize()
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)


def test_v12_mn_major_runs_v8(dev):
    ops = _ops()
    dy = _rand(1000, 904, dev=dev, seed=330)
    w = _rand(904, 600, dev=dev, seed=331, scale=0.05)
    assert torch.equal(ops.gemm(dy, w.t(), variant=26, split_k=1), ops.gemm(dy, w.t(), variant=24, split_k=1))
