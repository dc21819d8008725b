"""v11 GEMM (256x256 tiles of v8 on 32x32x16 MFMAs, K-major x K-major; forced variant 23,
variant 24 forces v8) against a torch fp32 reference of the same op, and against v8: the
two accumulate each k32 slice in a different MFMA shape, so they agree to fp32 rounding
(bf16 outputs within one ulp), not bit for bit.  Every epilogue the forward GEMMs use:
bias, GELU / SiLU, residual (row modulus), pre-activation aux, fp32 residual stream,
accumulate, alpha (x device scalar), the fused SwiGLU (bit-exact with v11 + k_swiglu_fwd), the
q|k|v scatter (bit-exact with v11 + k_qkv_split), split-K planes, partial tiles and K tails.
Tolerances as tests/test_gemm_gpu.py (fp32 accumulation, one bf16 rounding)."""
import pytest
import torch

from test_gemm_gpu import _check, _ops, _rand

pytestmark = pytest.mark.gpu

SHAPES = [(256, 256, 32), (512, 512, 256), (1458, 1152, 1152), (1000, 904, 600), (300, 272, 4304), (257, 520, 72),
          (6144 // 4, 4608, 3584 // 4), (128, 384, 4864)]


def _ulp_close(a, b):
    """bf16 tensors equal up to one unit in the last place (different fp32 summation orders)."""
    x, y = a.float(), b.float()
    ulp = torch.maximum(x.abs(), y.abs()) * 2.0 ** -7 + 1e-30
    return bool(((x - y).abs() <= ulp).all())


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_v11_forward_matches_fp32_and_v8(M, N, K, dev):
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=201)
    w = _rand(N, K, dev=dev, seed=202, scale=0.05)
    o11 = ops.gemm(a, w, variant=23, split_k=1)
    _check(o11, a.float() @ w.float().t())
    assert _ulp_close(o11, ops.gemm(a, w, variant=24, split_k=1))
    o32 = ops.gemm(a, w, variant=23, split_k=1, out_dtype=torch.float32)
    ref = a.float() @ w.float().t()
    assert float((o32 - ref).abs().max()) <= 1e-4 * float(ref.abs().max()) + 1e-4


@pytest.mark.parametrize("M,N,K", [(1458, 1152, 192), (600, 1152, 2304)])
def test_v11_epilogues(M, N, K, dev):
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=210)
    w = _rand(N, K, dev=dev, seed=211, scale=0.1)
    bias = _rand(N, dev=dev, seed=212)
    pos = _rand(729, N, dev=dev, seed=213)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    pre = a.float() @ w.float().t() + bias.float()
    rows = torch.arange(M, device=dev) % 729
    out = ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=pos, residual_row_mod=729, aux=aux, variant=23)
    _check(out, torch.nn.functional.gelu(pre, approximate="tanh") + pos.float()[rows])
    _check(aux, pre)
    for act, f in (("gelu_erf", torch.nn.functional.gelu), ("silu", torch.nn.functional.silu)):
        _check(ops.gemm(a, w, bias=bias, act=act, variant=23), f(pre))
    # fp32 residual stream (o_proj / fc2 / down_proj of an fp32 stream)
    g = torch.Generator(device=dev).manual_seed(214)
    res = torch.randn(M, N, generator=g, device=dev) * 3 + 1e-3
    o = ops.gemm(a, w, bias=bias, residual=res, out_dtype=torch.float32, variant=23, split_k=1)
    ref = pre + res
    assert float((o - ref).abs().max()) <= 2e-4 * float(ref.abs().max())
    # accumulate with alpha x device scalar (the lm_head wgrad form, here K-major)
    acc = torch.full((M, N), 2.0, device=dev)
    s = torch.tensor([2.0], device=dev)
    ops.gemm(a, w, out=acc, accumulate=True, variant=23, alpha=0.25, alpha_dev=s)
    assert float((acc - (2 + 0.5 * (a.float() @ w.float().t()))).abs().max()) < 1e-3


@pytest.mark.parametrize("split", [2, 3])
def test_v11_split_k(split, dev):
    ops = _ops()
    M, N, K = 520, 384, 2248
    a = _rand(M, K, dev=dev, seed=220)
    w = _rand(N, K, dev=dev, seed=221, scale=0.05)
    bias = _rand(N, dev=dev, seed=222)
    _check(ops.gemm(a, w, bias=bias, variant=23, split_k=split), a.float() @ w.float().t() + bias.float())


@pytest.mark.parametrize("M,I,K", [(300, 256, 96), (1536, 384, 896), (257, 128, 600), (512, 1280, 3584)])
def test_v11_swiglu_bitexact(M, I, K, dev):
    """act='swiglu' on v11 == v11's plain gate|up GEMM + k_swiglu_fwd, bit for bit."""
    ops = _ops()
    h = _rand(M, K, dev=dev, seed=230)
    w = _rand(2 * I, K, dev=dev, seed=231, scale=0.05)
    gu = ops.gemm(h, w, variant=23, split_k=1)
    aux = torch.empty(M, 2 * I, dtype=torch.bfloat16, device=dev)
    a = ops.gemm(h, w, act="swiglu", aux=aux, variant=23)
    assert torch.equal(aux, gu)
    assert torch.equal(a, ops.swiglu_fwd(gu, I))
    g = gu.float()
    _check(a, torch.nn.functional.silu(g[:, :I]) * g[:, I:])


@pytest.mark.parametrize("shape", ["teacher", "student", "siglip"])
def test_v11_qkv_scatter_bitexact(shape, dev):
    ops = _ops()
    B, S, K, nq, nkv, hd, hdp, rope = {
        "teacher": (1, 1536, 3584, 28, 4, 128, 128, True),
        "student": (2, 1536, 896, 14, 2, 64, 64, True),
        "siglip": (2, 729, 1152, 16, 16, 72, 96, False)}[shape]
    M, N = B * S, (nq + 2 * nkv) * hd
    x = _rand(M, K, dev=dev, seed=240)
    w = _rand(N, K, dev=dev, seed=241, scale=0.05)
    bias = _rand(N, dev=dev, seed=242)
    cos = sin = None
    if rope:
        inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
        f = torch.arange(S, dtype=torch.float32)[:, None] * inv[None]
        cos, sin = f.cos().to(dev).contiguous(), f.sin().to(dev).contiguous()
    q0, k0, v0 = ops.qkv_split(ops.gemm(x, w, bias=bias, variant=23, split_k=1), B, S, nq, nkv, hd, hdp, cos, sin)
    q = torch.full((B, nq, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)
    k = torch.full((B, nkv, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)
    v = torch.full((B, nkv, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)
    ops.gemm_qkv(x, w, bias, q, k, v, S, nq, nkv, hd, hdp, cos, sin, variant=23)
    torch.cuda.synchronize()
    for got, ref, n in ((q, q0, "q"), (k, k0, "k"), (v, v0, "v")):
        assert torch.equal(got, ref), f"{n}: {int((got != ref).sum())} elements differ"


def test_v11_mn_major_falls_back_to_v8(dev):
    """v11 is K-major x K-major only: forced on a dgrad / wgrad it runs v8 (same results)."""
    ops = _ops()
    dy = _rand(1000, 904, dev=dev, seed=250)
    w = _rand(904, 600, dev=dev, seed=251, scale=0.05)
    assert torch.equal(ops.gemm(dy, w.t(), variant=23, split_k=1), ops.gemm(dy, w.t(), variant=24, split_k=1))
