"""bf16 MFMA GEMM (kd_gemm) against a torch fp32 reference of the same op.

Tolerance: inputs are bf16; the kernel accumulates in fp32 and rounds the output to
bf16 once, so |err| <= 2^-8 * |ref| + K * 2^-20 * max|a||b| covers it; we use
rtol 1e-2 / atol 1e-2 * rms(ref) on bf16 outputs and 1e-4 relative on fp32 outputs.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops
    return ops


def _rand(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev, torch.bfloat16)


def _check(out, ref, rtol=1e-2):
    ref = ref.float()
    err = (out.float() - ref).abs()
    tol = rtol * ref.abs() + rtol * ref.pow(2).mean().sqrt()
    assert bool((err <= tol).all()), f"max err {err.max().item()} (rms ref {ref.pow(2).mean().sqrt().item()})"


SHAPES = [(128, 128, 64), (256, 384, 512), (1458, 1152, 1152), (100, 72, 4304), (6144 // 4, 896, 4864 // 2),
          (7, 13, 8), (129, 130, 72)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_forward_nt(M, N, K, dev):
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=1)
    w = _rand(N, K, dev=dev, seed=2, scale=0.05)
    out = ops.gemm(a, w)
    _check(out, a.float() @ w.float().t())


@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (1458, 1152, 1152), (1536, 896, 600)])
def test_dgrad_b_mn(M, N, K, dev):
    """dX = dY W  with W [N_out, K_in] read MN-major (no transpose copy)."""
    ops = _ops()
    dy = _rand(M, N, dev=dev, seed=3)
    w = _rand(N, K, dev=dev, seed=4, scale=0.05)   # weight [out=N, in=K]
    dx = ops.gemm(dy, w.t())                        # b = W^T view: [K, N] with stride (1, K)
    _check(dx, dy.float() @ w.float())


@pytest.mark.parametrize("M,N,K", [(384, 256, 512), (1152, 1152, 1458), (896, 4864, 1536)])
def test_wgrad_both_mn(M, N, K, dev):
    """dW[out, in] = dY^T X: a = dY^T (MN-major), b = X^T (MN-major), contraction over tokens."""
    ops = _ops()
    dy = _rand(K, M, dev=dev, seed=5)   # tokens x out
    x = _rand(K, N, dev=dev, seed=6)    # tokens x in
    dw = ops.gemm(dy.t(), x.t(), out_dtype=torch.float32)
    ref = dy.float().t() @ x.float()
    err = (dw - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item() + 1e-3


def test_a_mn_b_k(dev):
    ops = _ops()
    a = _rand(512, 256, dev=dev, seed=7)   # stored [K][M]
    b = _rand(320, 512, dev=dev, seed=8)
    out = ops.gemm(a.t(), b)
    _check(out, a.float().t() @ b.float().t())


def test_epilogue_bias_act_residual_aux_accumulate(dev):
    ops = _ops()
    M, N, K = 300, 200, 96
    a = _rand(M, K, dev=dev, seed=9)
    w = _rand(N, K, dev=dev, seed=10, scale=0.1)
    bias = _rand(N, dev=dev, seed=11)
    res = _rand(M, N, dev=dev, seed=12)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    pre = a.float() @ w.float().t() * 0.5 + bias.float()
    for act, f in (("gelu_tanh", lambda x: torch.nn.functional.gelu(x, approximate="tanh")),
                   ("gelu_erf", torch.nn.functional.gelu), ("silu", torch.nn.functional.silu)):
        out = ops.gemm(a, w, bias=bias, act=act, residual=res, aux=aux, alpha=0.5)
        _check(out, f(pre) + res.float())
        _check(aux, pre)
    acc = torch.ones(M, N, dtype=torch.float32, device=dev)
    ops.gemm(a, w, out=acc, accumulate=True)
    ref = 1 + a.float() @ w.float().t()
    assert (acc - ref).abs().max().item() < 1e-3 * ref.abs().max().item()
    s = torch.tensor([2.0], device=dev)
    out = ops.gemm(a, w, alpha_dev=s, alpha=0.25, out_dtype=torch.float32)
    assert (out - 0.5 * (a.float() @ w.float().t())).abs().max().item() < 1e-3
