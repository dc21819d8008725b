"""LayerNorm / RMSNorm forward A/B (KD_NORM_FWD_V=1: the previous kernel) bit-exact, moved from tests/test_layers_gpu.py (round 5).

Runs against the tools' A/B library, built with
    python knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd/csrc/build.py --ab
    python -m pytest tools/ab_tests -m gpu        (conftest.py points KDSTEP_LIB at tools/ab/libkdstep_ab.so)
The product library rejects these variants / ignores these switches.
"""
import pytest
import torch

from test_layers_gpu import _ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,D,rms,f32", [(6144, 3584, True, False), (5832, 1152, False, True), (6144, 896, True, True),
                                         (37, 200, False, False), (5, 4096, True, True), (3, 520, False, True)])
def test_norm_fwd_hoisted_loads_bitexact(R, D, rms, f32, dev):
    """k_norm_fwd2 (every load of a row issued first, chunk index clamped) == the previous
    k_norm_fwd (KD_NORM_FWD_V=1) bit for bit: y, mean and rstd; ragged D (partial last chunk round)."""
    import os
    ops = _ops()
    g = torch.Generator(device=dev).manual_seed(R + D)
    x = torch.randn(R, D, device=dev, generator=g)
    x = x if f32 else x.bfloat16()
    w = torch.randn(D, device=dev, generator=g).bfloat16()
    b = None if rms else torch.randn(D, device=dev, generator=g).bfloat16()
    outs = []
    try:
        for var in ("1", "2"):
            os.environ["KD_NORM_FWD_V"] = var
            outs.append(ops.norm_fwd(x, w, b, 1e-6, rms=rms, save_stats=True))
    finally:
        os.environ.pop("KD_NORM_FWD_V", None)
    (y0, m0, r0), (y1, m1, r1) = outs
    assert torch.equal(y0, y1) and torch.equal(r0, r1)
    assert (m0 is None and m1 is None) or torch.equal(m0, m1)
