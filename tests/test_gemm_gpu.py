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


@pytest.mark.parametrize("variant,split_k", [(1, 1), (5, 1), (6, 1), (7, 1), (16, 1), (16, 3), (0, 0), (21, 0), (32, 3)])
def test_fp32_residual_stream(variant, split_k, dev):
    """C (fp32) = A B^T + bias + residual (fp32): the fp32 residual stream's epilogue (o_proj /
    fc2 / down_proj with kd_model_set_residual_f32) in every kernel and through the split-K
    reduce; the residual is added in fp32, not rounded to bf16."""
    ops = _ops()
    M, N, K = 600, 1152, 2304
    a = _rand(M, K, dev=dev, seed=21)
    w = _rand(N, K, dev=dev, seed=22, scale=0.05)
    bias = _rand(N, dev=dev, seed=23)
    g = torch.Generator(device=dev).manual_seed(24)
    res = torch.randn(M, N, generator=g, device=dev) * 3 + 1e-3   # fp32 values off the bf16 grid
    out = ops.gemm(a, w, bias=bias, residual=res, out_dtype=torch.float32, variant=variant, split_k=split_k)
    ref = a.float() @ w.float().t() + bias.float() + res
    err = (out - ref).abs()
    assert float(err.max()) <= 2e-4 * float(ref.abs().max()), float(err.max())
    # bf16 rounding of the residual alone would be off by up to |res| * 2^-9
    assert float((out - (a.float() @ w.float().t() + bias.float() + res.bfloat16().float())).abs().max()) > 1e-3
    with pytest.raises(RuntimeError, match="fp32 residual"):
        ops.gemm(a, w, residual=res)   # bf16 C with an fp32 residual is rejected


VARIANTS = [1, 5, 6, 7, 16]   # 128x128 v1; v3 256x256 / 256x128 / 128x256 (8 waves); v8 256x256 (4 waves, AGPR acc);
#                                  v9 256x256 (8 waves, ping-pong)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (1458, 1152, 1152), (1000, 904, 600), (300, 272, 4304)])
def test_variants_all_layouts(variant, M, N, K, dev):
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=31)
    w = _rand(N, K, dev=dev, seed=32, scale=0.05)
    _check(ops.gemm(a, w, variant=variant), a.float() @ w.float().t())
    # dgrad: dX[M, K] = dY[M, N] W[N, K]
    dy = _rand(M, N, dev=dev, seed=33)
    _check(ops.gemm(dy, w.t(), variant=variant), dy.float() @ w.float())
    if K % 8:
        return
    # wgrad: dW[N, K] = dY^T X over M tokens (fp32 accumulate)
    acc = torch.ones(N, K, dtype=torch.float32, device=dev)
    ops.gemm(dy.t(), a.t(), out=acc, accumulate=True, variant=variant)
    ref = 1 + dy.float().t() @ a.float()
    assert (acc - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-3
    # A MN-major x B K-major (MN-major operands need rows % 8 == 0)
    if M % 8 == 0:
        at = _rand(K, M, dev=dev, seed=34)
        _check(ops.gemm(at.t(), w, variant=variant), at.float().t() @ w.float().t())


@pytest.mark.parametrize("variant", [5, 6, 7, 16])
def test_variant_epilogue(variant, dev):
    ops = _ops()
    M, N, K = 1458, 1152, 192
    a = _rand(M, K, dev=dev, seed=40)
    w = _rand(N, K, dev=dev, seed=41, scale=0.1)
    bias = _rand(N, dev=dev, seed=42)
    pos = _rand(729, N, dev=dev, seed=43)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    pre = a.float() @ w.float().t() + bias.float()
    out = ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=pos, residual_row_mod=729, aux=aux, variant=variant)
    ref = torch.nn.functional.gelu(pre, approximate="tanh") + pos.float().repeat(2, 1)
    _check(out, ref)
    _check(aux, pre)
    o32 = torch.full((M, N), 2.0, device=dev)
    ops.gemm(a, w, out=o32, accumulate=True, variant=variant, alpha=0.5)
    assert (o32 - (2 + 0.5 * (a.float() @ w.float().t()))).abs().max().item() < 1e-3


@pytest.mark.parametrize("split", [2, 3, 7])
@pytest.mark.parametrize("variant", [0, 6, 7, 16, 32])
@pytest.mark.parametrize("M,N,K", [(520, 384, 2248), (1152, 1152, 5832)])
def test_splitk_all_layouts(split, variant, M, N, K, dev):
    """Forced K splits (fp32 partial planes + reduce; variant 32: v8 with the in-launch fold) in
    every operand layout; K is not a multiple of split*32, so the last split is ragged."""
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=50)
    w = _rand(N, K, dev=dev, seed=51, scale=0.05)
    _check(ops.gemm(a, w, variant=variant, split_k=split), a.float() @ w.float().t())
    at = _rand(K, M, dev=dev, seed=52)
    _check(ops.gemm(at.t(), w, variant=variant, split_k=split), at.float().t() @ w.float().t())
    wt = _rand(K, N, dev=dev, seed=53, scale=0.05)
    _check(ops.gemm(a, wt.t(), variant=variant, split_k=split), a.float() @ wt.float())
    acc = torch.ones(M, N, dtype=torch.float32, device=dev)
    ops.gemm(at.t(), wt.t(), out=acc, accumulate=True, variant=variant, split_k=split)
    ref = 1 + at.float().t() @ wt.float()
    assert (acc - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-3


@pytest.mark.parametrize("M,N,K", [(1152, 1152, 5832), (1000, 904, 4296), (6144, 5632, 256), (6144, 4608, 3584),
                                   (5832, 1152, 4304)])
def test_stream_k_all_layouts(M, N, K, dev):
    """Stream-K (variant 21): all but the last whole wave of 256 x 256 tiles run data-parallel (the
    528- and 432-tile cases), then 256 workgroups take equal runs of the remaining tiles' k-steps;
    a tile shared by several runs is folded inside the launch by its last-arriving piece, tiles a
    single run covers get the epilogue directly. Ragged M / N / K tails; every operand layout; fp32 +=."""
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=60)
    w = _rand(N, K, dev=dev, seed=61, scale=0.05)
    _check(ops.gemm(a, w, variant=21), a.float() @ w.float().t())
    wt = _rand(K, N, dev=dev, seed=63, scale=0.05)
    _check(ops.gemm(a, wt.t(), variant=21), a.float() @ wt.float())
    if M % 8 == 0:
        at = _rand(K, M, dev=dev, seed=62)
        _check(ops.gemm(at.t(), w, variant=21), at.float().t() @ w.float().t())
        acc = torch.ones(M, N, dtype=torch.float32, device=dev)
        ops.gemm(at.t(), wt.t(), out=acc, accumulate=True, variant=21)
        ref = 1 + at.float().t() @ wt.float()
        assert (acc - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-3


def test_stream_k_epilogue(dev):
    """The stream-K fold and the direct tiles apply the whole epilogue: alpha * alpha_dev,
    bias, aux, act, residual (row mod), bf16 accumulate."""
    ops = _ops()
    M, N, K = 1458, 1152, 4304
    a = _rand(M, K, dev=dev, seed=64)
    w = _rand(N, K, dev=dev, seed=65, scale=0.02)
    bias = _rand(N, dev=dev, seed=66)
    pos = _rand(729, N, dev=dev, seed=67)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    s = torch.tensor([0.5], device=dev)
    pre = 0.5 * 2.0 * (a.float() @ w.float().t()) + bias.float()
    out = ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=pos, residual_row_mod=729, aux=aux, alpha=2.0,
                   alpha_dev=s, variant=21)
    _check(out, torch.nn.functional.gelu(pre, approximate="tanh") + pos.float().repeat(2, 1))
    _check(aux, pre)
    o = _rand(M, N, dev=dev, seed=68)
    ref = o.float() + a.float() @ w.float().t()
    ops.gemm(a, w, out=o, accumulate=True, variant=21)
    _check(o, ref)


@pytest.mark.parametrize("M,N,K", [(6144, 3584, 3584), (1458, 1152, 4304), (6144, 896, 4864)])
def test_stream_k_fold_is_deterministic(M, N, K, dev):
    """The in-launch fold sums a shared tile's pieces in piece order whichever piece arrives last:
    repeated launches (with another stream's GEMM competing for the CUs in the second round) give
    the same bits; and the result matches the fp32 reference."""
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=70)
    w = _rand(N, K, dev=dev, seed=71, scale=0.05)
    ref = ops.gemm(a, w, variant=21)
    _check(ref, a.float() @ w.float().t())
    for _ in range(3):
        assert torch.equal(ops.gemm(a, w, variant=21), ref)
    side = torch.cuda.Stream(device=dev)
    x = _rand(4096, 4096, dev=dev, seed=72)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(4):
            y = x @ x
    out = ops.gemm(a, w, variant=21)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    del y


def test_splitk_epilogue(dev):
    """The reduce pass applies the whole epilogue: alpha * alpha_dev, bias, aux, act,
    residual (row mod), bf16 accumulate."""
    ops = _ops()
    M, N, K = 1458, 1152, 3072
    a = _rand(M, K, dev=dev, seed=60, scale=0.2)
    w = _rand(N, K, dev=dev, seed=61, scale=0.02)
    bias = _rand(N, dev=dev, seed=62)
    pos = _rand(729, N, dev=dev, seed=63)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    ad = torch.tensor([0.75], device=dev)
    pre = 1.5 * 0.75 * (a.float() @ w.float().t()) + bias.float()
    out = ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=pos, residual_row_mod=729, aux=aux, alpha=1.5,
                   alpha_dev=ad, split_k=3)
    _check(out, torch.nn.functional.gelu(pre, approximate="tanh") + pos.float().repeat(2, 1))
    _check(aux, pre)
    base = _rand(M, N, dev=dev, seed=64)
    o = base.clone()
    ops.gemm(a, w, out=o, accumulate=True, split_k=4)
    _check(o, base.float() + a.float() @ w.float().t())


@pytest.mark.parametrize("M,N,K", [(896, 896, 6144), (3456, 1152, 5832), (1152, 4304, 5832)])
def test_splitk_auto_wgrad(M, N, K, dev):
    """The cost model's own choice on the step's weight-gradient shapes (MN x MN, fp32 +=)."""
    ops = _ops()
    dy = _rand(K, M, dev=dev, seed=70)
    x = _rand(K, N, dev=dev, seed=71)
    acc = torch.full((M, N), 0.5, dtype=torch.float32, device=dev)
    ops.gemm(dy.t(), x.t(), out=acc, accumulate=True)
    ref = 0.5 + dy.float().t() @ x.float()
    assert (acc - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-3


def test_hybrid_split_tail(dev):
    """Auto plan on a GEMM just over one wave of tiles: whole waves run unsplit with the
    kernel epilogue, the tail tiles split-K with the reduce epilogue; both must give the
    full epilogue (alpha, bias, aux, act, residual) and fp32 accumulate in every layout."""
    ops = _ops()
    M, N, K = 4608, 3840, 4096
    a = _rand(M, K, dev=dev, seed=80, scale=0.2)
    w = _rand(N, K, dev=dev, seed=81, scale=0.02)
    bias = _rand(N, dev=dev, seed=82)
    res = _rand(M, N, dev=dev, seed=83)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    var, split, dp = ops.gemm_plan(a, w)
    assert split > 1 and 0 < dp < 18 * 15, (var, split, dp)
    pre = 1.25 * (a.float() @ w.float().t()) + bias.float()
    out = ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=res, aux=aux, alpha=1.25)
    _check(out, torch.nn.functional.gelu(pre, approximate="tanh") + res.float())
    _check(aux, pre)
    at = _rand(K, M, dev=dev, seed=84)
    wt = _rand(K, N, dev=dev, seed=85, scale=0.05)
    for A, B, ref in ((a, wt.t(), a.float() @ wt.float()), (at.t(), wt.t(), at.float().t() @ wt.float()),
                      (at.t(), w, at.float().t() @ w.float().t())):
        acc = torch.full((M, N), 0.5, dtype=torch.float32, device=dev)
        assert ops.gemm_plan(A, B, out=acc, accumulate=True)[2] > 0
        ops.gemm(A, B, out=acc, accumulate=True)
        r = 0.5 + ref
        assert (acc - r).abs().max().item() <= 1e-4 * r.abs().max().item() + 1e-3


@pytest.mark.parametrize("M,I,K", [(300, 256, 96), (1536, 384, 896), (257, 128, 600), (512, 1280, 3584)])
def test_swiglu_epilogue_bitexact(M, I, K, dev):
    """act='swiglu' (gate|up GEMM + silu(gate)*up fused, v8) == the unfused GEMM + k_swiglu_fwd,
    bit for bit (same accumulation order, same bf16 rounding of gate/up, same fp32 formula);
    aux carries the [M, 2I] pre-activation the backward reads."""
    ops = _ops()
    h = _rand(M, K, dev=dev, seed=21)
    w = _rand(2 * I, K, dev=dev, seed=22, scale=0.05)
    gu_ref = ops.gemm(h, w, variant=16, split_k=1)
    a_ref = ops.swiglu_fwd(gu_ref, I)
    aux = torch.empty(M, 2 * I, dtype=torch.bfloat16, device=dev)
    a = ops.gemm(h, w, act="swiglu", aux=aux)
    assert a.shape == (M, I)
    assert torch.equal(aux, gu_ref)
    assert torch.equal(a, a_ref)
    assert torch.equal(ops.gemm(h, w, act="swiglu"), a_ref)
    # alpha != 1 takes the scaled staging path of the epilogue (alpha == 1 skips the multiply)
    half = ops.gemm(h, w, alpha=0.5, variant=16, split_k=1)
    assert torch.equal(ops.gemm(h, w, act="swiglu", alpha=0.5), ops.swiglu_fwd(half, I))
    g = gu_ref.float()
    _check(a, torch.nn.functional.silu(g[:, :I]) * g[:, I:])


@pytest.mark.parametrize("variant", [0, 5, 6, 7, 16, 21])
@pytest.mark.parametrize("M, N, K", [(1100, 1040, 392), (6144 // 2, 4864, 896), (5832 // 4, 4304, 1152)])
def test_fused_backward_activation(variant, M, N, K, dev):
    """KD_ACT_DGELU_TANH / KD_ACT_DSWIGLU: the dgrad GEMM with the activation backward in its
    epilogue equals the unfused GEMM (no split) followed by k_act_bwd / k_swiglu_bwd bit for
    bit (the SigLIP fc2 dgrad and the Qwen2 down-proj dgrad of the student backward)."""
    ops = _ops()
    dy = _rand(M, K, dev=dev, seed=41)
    w = _rand(K, N, dev=dev, seed=42, scale=K ** -0.5)
    v = ops.gemm(dy, w.t(), variant=variant, split_k=1 if variant != 21 else 0)
    pre = _rand(M, N, dev=dev, seed=43)
    out = ops.gemm(dy, w.t(), act="dgelu_tanh", aux=pre, variant=variant)
    assert torch.equal(out, ops.act_bwd(pre, v, "gelu_tanh"))
    gu = _rand(M, 2 * N, dev=dev, seed=44)
    out2 = ops.gemm(dy, w.t(), act="dswiglu", aux=gu, variant=variant)
    assert out2.shape == (M, 2 * N)
    assert torch.equal(out2, ops.swiglu_bwd(gu, v, N))
    # and against torch autograd of the activations (fp32 math on the same bf16 operands)
    x = pre.float().requires_grad_(True)
    torch.nn.functional.gelu(x, approximate="tanh").backward(v.float())
    _check(out, x.grad)


@pytest.mark.parametrize("shape,variant", [
    ("teacher", 0), ("teacher", 16), ("teacher", 6), ("teacher", 21), ("student", 0), ("student", 5), ("student", 7),
    ("siglip", 0), ("siglip", 16), ("siglip", 6), ("siglip", 21)])
def test_qkv_scatter_epilogue_equals_gemm_then_split(shape, variant, dev):
    """The fused q|k|v projection (kd_qkv_scatter epilogue: bias, bf16 rounding, head-major
    scatter, RoPE on q / k, zeroed padding) equals the plain GEMM followed by k_qkv_split bit
    for bit, in every tiled kernel: the Qwen2-7B (28q / 4kv, hd 128), Qwen2-0.5B (14q / 2kv,
    hd 64) and SigLIP (16 heads, hd 72 padded to 96, no RoPE) attention inputs."""
    ops = _ops()
    B, S, K, nq, nkv, hd, hdp, rope = {
        "teacher": (2, 1536, 3584, 28, 4, 128, 128, True),
        "student": (2, 1536, 896, 14, 2, 64, 64, True),
        "siglip": (4, 729, 1152, 16, 16, 72, 96, False)}[shape]
    M, N = B * S, (nq + 2 * nkv) * hd
    x = _rand(M, K, dev=dev, seed=31)
    w = _rand(N, K, dev=dev, seed=32, scale=0.05)
    bias = _rand(N, dev=dev, seed=33)
    cos = sin = None
    if rope:
        inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
        f = torch.arange(S, dtype=torch.float32)[:, None] * inv[None]
        cos, sin = f.cos().to(dev).contiguous(), f.sin().to(dev).contiguous()
    qkv = ops.gemm(x, w, bias=bias, variant=variant, split_k=1 if variant != 21 else 0)
    q0, k0, v0 = ops.qkv_split(qkv, B, S, nq, nkv, hd, hdp, cos, sin)
    q = torch.full((B, nq, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)   # garbage: the padding must be zeroed
    k = torch.full((B, nkv, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)
    v = torch.full((B, nkv, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)
    ops.gemm_qkv(x, w, bias, q, k, v, S, nq, nkv, hd, hdp, cos, sin, variant=variant)
    torch.cuda.synchronize()
    for got, ref, n in ((q, q0, "q"), (k, k0, "k"), (v, v0, "v")):
        assert torch.equal(got, ref), f"{n}: {int((got != ref).sum())} elements differ"


@pytest.mark.parametrize("M,I,K", [(6144, 4864, 896), (2048, 3584, 1536)])
def test_stream_k_swiglu_matches_plain_stream_k(M, I, K, dev):
    """The SwiGLU build on stream-K (variant 21: 912 / 224 gate|up tiles, a data-parallel prefix
    and runs folded in-launch): silu(gate) * up of the pre-activations the plain stream-K GEMM
    of the same gathered tiles produces, and the aux output equals that GEMM bit for bit."""
    ops = _ops()
    h = _rand(M, K, dev=dev, seed=81)
    w = _rand(2 * I, K, dev=dev, seed=82, scale=K ** -0.5)
    aux = torch.empty(M, 2 * I, dtype=torch.bfloat16, device=dev)
    a = ops.gemm(h, w, act="swiglu", aux=aux, variant=21)
    g = (h.float() @ w.float().t())
    _check(aux, g)
    _check(a, torch.nn.functional.silu(aux.float()[:, :I]) * aux.float()[:, I:])
    assert torch.equal(ops.gemm(h, w, act="swiglu", aux=aux, variant=21), a)   # deterministic


@pytest.mark.parametrize("M,N,K,split", [(896, 896, 6144, 8), (1152, 4304, 5832, 3), (6144, 3584, 3584, 0)])
def test_splitk_fold_equals_reduce(M, N, K, split, dev):
    """Variant 32 (v8 split-K folded in-launch by each tile's last-arriving split) sums the S pieces
    in split order like the reduce launch (x0 + x1 + ...): the same fp32 sums, and the same result
    through the whole epilogue (fp32 += here; split 0: the cost model's plan, the hybrid tail).
    Deterministic whichever split arrives last."""
    ops = _ops()
    a = _rand(K, M, dev=dev, seed=91)
    b = _rand(K, N, dev=dev, seed=92, scale=0.05)
    ref = torch.ones(M, N, dtype=torch.float32, device=dev)
    ops.gemm(a.t(), b.t(), out=ref, accumulate=True, variant=16, split_k=split)
    for _ in range(2):
        got = torch.ones(M, N, dtype=torch.float32, device=dev)
        ops.gemm(a.t(), b.t(), out=got, accumulate=True, variant=32, split_k=split)
        assert torch.equal(got, ref), float((got - ref).abs().max())
