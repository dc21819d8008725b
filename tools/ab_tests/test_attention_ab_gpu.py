"""Attention A/B variants (KD_ATTN_FWD_V, KD_ATTN_BWD_V) against the product kernels, moved from tests/test_attention_gpu.py (round 5).

Runs against the tools' A/B library, built with
    python knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd/csrc/build.py --ab
    python -m pytest tools/ab_tests -m gpu        (conftest.py points KDSTEP_LIB at tools/ab/libkdstep_ab.so)
The product library rejects these variants / ignores these switches.
"""
import pytest
import torch

from test_attention_gpu import CASES, _inputs, _ops, _ref_pabs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["16", "32"])
@pytest.mark.parametrize("B,H,HKV,S,hd,hdp,causal", [CASES[1], CASES[2], CASES[3], CASES[7], CASES[8]])
def test_attn_fwd_variants_agree(B, H, HKV, S, hd, hdp, causal, variant, dev):
    """The pipelined 32x32x16 kernel (default), the unpipelined one (KD_ATTN_FWD_V=32) and the
    16x16x32 one (=16) compute the same softmax; they differ only in the fp32 summation order
    of the scores / row sums and the sub-tile width of the lazy rescale (which changes the
    bf16 rounding of P): outputs within 2^-7 (|o| + P|V|), lse within 1e-5 relative."""
    import os
    ops = _ops()
    q, k, v = _inputs(B, H, HKV, S, hd, hdp, dev)
    outs = []
    try:
        for var in ("0", variant):
            os.environ["KD_ATTN_FWD_V"] = var   # read by the launcher on every call
            outs.append(ops.attn_fwd(q, k, v, hd, causal))
    finally:
        os.environ.pop("KD_ATTN_FWD_V", None)
    (o0, l0), (o1, l1) = outs
    d = (o0.float() - o1.float()).abs()
    pabs = _ref_pabs(q[..., :hd].float(), k[..., :hd].float(), v[..., :hd].float(), causal, hd).permute(0, 2, 1, 3)
    assert bool((d <= 2.0 ** -7 * (o0.float().abs() + pabs) + 1e-4).all()), d.max().item()
    assert (l0 - l1).abs().max().item() <= 1e-5 * l0.abs().max().item() + 1e-5


@pytest.mark.parametrize("B,H,HKV,S,hd,hdp,causal", [CASES[0], CASES[1], CASES[3], CASES[4], CASES[5], CASES[6]])
def test_attn_bwd_dkdv_variants_bitexact(B, H, HKV, S, hd, hdp, causal, dev):
    """The round-6 16x16x32 dK / dV with two 16-key sub-tiles per wave (KD_ATTN_BWD_V=2) == the
    one-sub-tile kernel (KD_ATTN_BWD_V=16) bit for bit: the same MFMA sequence and arithmetic per
    element; only the sharing of LDS fragments between the sub-tiles differs (and fully masked
    causal query halves are skipped, which adds exact zeros). (The product default is the 32x32x16
    pair, held against the fp32 reference by tests/test_attention_gpu.py.)"""
    import os
    ops = _ops()
    q, k, v = _inputs(B, H, HKV, S, hd, hdp, dev, seed=4)
    o, lse = ops.attn_fwd(q, k, v, hd, causal)
    g = torch.Generator().manual_seed(5)
    do = torch.randn(B, S, H, hd, generator=g).to(dev, torch.bfloat16)
    outs = []
    try:
        for var in ("2", "16"):
            os.environ["KD_ATTN_BWD_V"] = var
            outs.append(ops.attn_bwd(q, k, v, o, do, lse, hd, causal))
    finally:
        os.environ.pop("KD_ATTN_BWD_V", None)
    (dq0, dk0, dv0), (dq1, dk1, dv1) = outs
    sl = (Ellipsis, slice(0, hd))   # the head-dim padding [hd, hdp) is not an output
    assert torch.equal(dk0[sl], dk1[sl]) and torch.equal(dv0[sl], dv1[sl]) and torch.equal(dq0[sl], dq1[sl])


@pytest.mark.parametrize("B,H,HKV,S,hd,hdp,causal", CASES)
def test_attn_fwd_six_waves_bitexact(B, H, HKV, S, hd, hdp, causal, dev):
    """Forced variant 36: workgroups of six waves (192 query rows; only waves 0-3 stage K/V) ==
    the four-wave kernel bit for bit: every wave walks its own queries over the same K/V tiles
    in the same order (causal: the same per-wave tile count).  Head dim 128 keeps four waves."""
    import os
    ops = _ops()
    q, k, v = _inputs(B, H, HKV, S, hd, hdp, dev, seed=3)
    outs = []
    try:
        for var in ("32", "36"):
            os.environ["KD_ATTN_FWD_V"] = var
            outs.append(ops.attn_fwd(q, k, v, hd, causal))
    finally:
        os.environ.pop("KD_ATTN_FWD_V", None)
    (o0, l0), (o1, l1) = outs
    assert torch.equal(o0, o1) and torch.equal(l0, l1)


@pytest.mark.parametrize("B,H,HKV,S,hd,hdp,causal", CASES)
def test_attn_fwd_two_blocks_per_wave_bitexact(B, H, HKV, S, hd, hdp, causal, dev):
    """Forced variant 64 (k_attn_fwd64): two 32-row query blocks per wave sharing every K / V^T
    fragment read, 256 query rows per workgroup == the four-wave k_attn_fwd32 bit for bit (per
    query row the same operations in the same order; a wave's two causal blocks end on one tile)."""
    import os
    ops = _ops()
    q, k, v = _inputs(B, H, HKV, S, hd, hdp, dev, seed=4)
    outs = []
    try:
        for var in ("32", "64"):
            os.environ["KD_ATTN_FWD_V"] = var
            outs.append(ops.attn_fwd(q, k, v, hd, causal))
    finally:
        os.environ.pop("KD_ATTN_FWD_V", None)
    (o0, l0), (o1, l1) = outs
    assert torch.equal(o0, o1) and torch.equal(l0, l1)
