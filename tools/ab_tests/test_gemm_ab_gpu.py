"""GEMM A/B builds (v9 = variant 20, register staging = variant 22) bit-exact against v8, moved from tests/test_gemm_gpu.py (round 5).

Runs against the tools' A/B library, built with
    python knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd/csrc/build.py --ab
    python -m pytest tools/ab_tests -m gpu        (conftest.py points KDSTEP_LIB at tools/ab/libkdstep_ab.so)
The product library rejects these variants / ignores these switches.
"""
import pytest
import torch

from test_gemm_gpu import _ops, _rand

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(6144 // 4, 896, 4864 // 2), (1456, 1152, 1152), (304, 520, 600), (4096, 4096, 4096)])
def test_v9_bitexact_vs_v8(M, N, K, dev):
    """v9 (8-wave ping-pong) accumulates every output element over the same k32 MFMA
    sequence as v8, so the two agree bit for bit in every operand layout, with and without
    the SwiGLU epilogue."""
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=90)
    w = _rand(N, K, dev=dev, seed=91, scale=0.05)
    at = _rand(K, M, dev=dev, seed=92)
    wt = _rand(K, N, dev=dev, seed=93, scale=0.05)
    for A, B in ((a, w), (a, wt.t()), (at.t(), w), (at.t(), wt.t())):
        assert torch.equal(ops.gemm(A, B, variant=20, split_k=1), ops.gemm(A, B, variant=16, split_k=1))
    if N % 256 == 0:
        g9 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        g8 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        o9 = ops.gemm(a, w, act="swiglu", aux=g9, variant=20)
        o8 = ops.gemm(a, w, act="swiglu", aux=g8, variant=16)
        assert torch.equal(o9, o8) and torch.equal(g9, g8)


@pytest.mark.parametrize("M,N,K", [(6144 // 4, 896, 4864 // 2), (1456, 1152, 1152), (304, 520, 600), (4096, 4096, 4096),
                                   (5832 // 4, 4304, 1152), (512, 512, 2248), (256, 768, 32), (300, 272, 4304)])
def test_register_staged_v8_bitexact(M, N, K, dev):
    """The register-staged v8 build (variant 22: buffer loads to VGPRs + ds_write_b128 instead of
    LDS-DMA, the same LDS image) accumulates over the same k32 MFMA sequence as v8: bit for bit
    equal, plain and with the epilogue (bias, gelu, residual, aux) and the SwiGLU build; K tails
    of every length, partial tiles, K shorter than the prefetch ring."""
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=120)
    w = _rand(N, K, dev=dev, seed=121, scale=0.05)
    assert torch.equal(ops.gemm(a, w, variant=22, split_k=1), ops.gemm(a, w, variant=16, split_k=1))
    bias = _rand(N, dev=dev, seed=122)
    res = _rand(M, N, dev=dev, seed=123)
    ax16 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    ax22 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    o16 = ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=res, aux=ax16, variant=16, split_k=1)
    o22 = ops.gemm(a, w, bias=bias, act="gelu_tanh", residual=res, aux=ax22, variant=22, split_k=1)
    assert torch.equal(o22, o16) and torch.equal(ax22, ax16)
    if N % 256 == 0:
        g16 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        g22 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        s16 = ops.gemm(a, w, act="swiglu", aux=g16, variant=16)
        s22 = ops.gemm(a, w, act="swiglu", aux=g22, variant=22)
        assert torch.equal(s22, s16) and torch.equal(g22, g16)


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 4096), (6144, 1024, 3584), (3000, 1280, 1152), (2048, 768, 600)])
def test_v8_stagger_matches_unstaggered(M, N, K, dev):
    """The k-loop stagger (KD_GEMM_STAGGER, the product default) only rotates where each tile's
    K loop starts: the same products, summed in another order -- equal to the unstaggered v8
    within fp32 reordering (bf16 outputs: at most a few 1-ulp differences), bit-identical where
    no tile rotates (one row group, K % 32 != 0 or K < 2048), and the same bits for the SwiGLU build's
    aux, pre-tiled B and the plain GEMM under the stagger."""
    import os
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=130)
    w = _rand(N, K, dev=dev, seed=131, scale=0.05)
    ref = ops.gemm(a, w, variant=16, split_k=1)
    os.environ["KD_GEMM_STAGGER"] = "1"
    try:
        got = ops.gemm(a, w, variant=16, split_k=1)
        if K % 32 or K < 2048:
            assert torch.equal(got, ref)
        d = (got.float() - ref.float()).abs()
        assert d.max().item() <= 2 ** -6 * ref.float().abs().max().item()
        assert (got != ref).float().mean().item() < 0.05
        assert torch.equal(ops.gemm(a, w, b_pretiled=ops.pretile_b(w)), got)
        if N % 256 == 0:
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            o = ops.gemm(a, w, act="swiglu", aux=aux)
            assert torch.equal(aux, got)
            assert torch.equal(o, ops.swiglu_fwd(got, N // 2))
    finally:
        os.environ["KD_GEMM_STAGGER"] = "0"


@pytest.mark.parametrize("M,N,K", [(5832, 4304, 1152), (5832, 1152, 4304), (300, 264, 96), (1100, 1040, 392),
                                   (6144, 896, 4864), (2048, 640, 2304), (257, 136, 40)])
def test_v8n_bitexact_vs_v8(M, N, K, dev, monkeypatch):
    """v8n (variant 30: 256x128 tiles, two workgroups per CU) runs v8's k32 MFMA sequence for every
    output element with v8's k-loop stagger row groups, so C is v8's bit for bit -- plain and with
    each epilogue it takes (bias + GELU-tanh + pre-activation aux, residual, fp32 accumulate);
    partial tiles, K tails shorter than a stage and than the ring, K >= 2048 (stagger on).  The
    reference is v8 over pre-tiled B (v8 at every size: a forced variant 16 runs v1 below 2^20
    outputs), bit-identical to plain v8 (tests/test_gemm_pretiled_gpu.py)."""
    monkeypatch.setenv("KD_GEMM_STAGGER", "1")   # the product default (the A/B suite runs v8 unstaggered)
    ops = _ops()
    a = _rand(M, K, dev=dev, seed=140)
    w = _rand(N, K, dev=dev, seed=141, scale=0.05)
    pt = ops.pretile_b(w)
    assert torch.equal(ops.gemm(a, w, variant=30), ops.gemm(a, w, b_pretiled=pt))
    bias = _rand(N, dev=dev, seed=142)
    res = _rand(M, N, dev=dev, seed=143)
    ax = [torch.empty(M, N, dtype=torch.bfloat16, device=dev) for _ in range(2)]
    o0 = ops.gemm(a, w, bias=bias, act="gelu_tanh", aux=ax[0], variant=30)
    o1 = ops.gemm(a, w, bias=bias, act="gelu_tanh", aux=ax[1], b_pretiled=pt)
    assert torch.equal(o0, o1) and torch.equal(ax[0], ax[1])
    assert torch.equal(ops.gemm(a, w, residual=res, variant=30), ops.gemm(a, w, residual=res, b_pretiled=pt))
    acc = [torch.full((M, N), 0.25, dtype=torch.float32, device=dev) for _ in range(2)]
    ops.gemm(a, w, out=acc[0], accumulate=True, variant=30)
    ops.gemm(a, w, out=acc[1], accumulate=True, b_pretiled=pt)
    assert torch.equal(acc[0], acc[1])


@pytest.mark.parametrize("B,S,K,nq,nkv,hd,hdp,rope", [(4, 1536, 3584, 28, 4, 128, 128, True),
                                                       (4, 1536, 896, 14, 2, 64, 64, True),
                                                       (8, 729, 1152, 16, 16, 72, 96, False)])
def test_v8n_qkv_scatter_bitexact_vs_v8(B, S, K, nq, nkv, hd, hdp, rope, dev, monkeypatch):
    """v8n's q|k|v scatter epilogue (128-column tiles: whole heads with RoPE, any split without) writes
    v8's head-major q / k / v bit for bit on the step's three attention-input shapes."""
    monkeypatch.setenv("KD_GEMM_STAGGER", "1")   # the product default (the A/B suite runs v8 unstaggered)
    ops = _ops()
    g = torch.Generator(device=dev).manual_seed(3)
    M, N = B * S, (nq + 2 * nkv) * hd
    x = torch.randn(M, K, generator=g, device=dev).bfloat16()
    w = (torch.randn(N, K, generator=g, device=dev) * K ** -0.5).bfloat16()
    bias = torch.randn(N, generator=g, device=dev).bfloat16()
    cos = sin = None
    if rope:
        inv = 1.0 / (1e6 ** (torch.arange(0, hd, 2, dtype=torch.float32, device=dev) / hd))
        fr = torch.arange(S, dtype=torch.float32, device=dev)[:, None] * inv[None]
        cos, sin = fr.cos().contiguous(), fr.sin().contiguous()
    outs = []
    for v in (30, 24):
        q = torch.full((B, nq, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)
        k = torch.full((B, nkv, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)
        vv = torch.full((B, nkv, S, hdp), 7.0, dtype=torch.bfloat16, device=dev)
        ops.gemm_qkv(x, w, bias, q, k, vv, S, nq, nkv, hd, hdp, cos, sin, variant=v)
        outs.append((q, k, vv))
    torch.cuda.synchronize()
    for a, b, n in zip(outs[0], outs[1], "qkv"):
        assert torch.equal(a, b), f"{n}: {int((a != b).sum())} elements differ"
