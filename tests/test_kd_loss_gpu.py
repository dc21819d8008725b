"""Parity of the fused HIP KD-loss kernel (kd_loss_fwd_bwd) with the reference.

Expected values come from the reference's own loss functions (tests/golden/kd_*.npz,
made by make_golden.py); inputs are regenerated from seeds and fed to the kernel as
bf16 (they are bf16-representable, so the kernel sees exactly the reference's values).

Tolerances (fp32 math in the kernel vs fp32 PyTorch in the reference):
  loss terms   rel 1e-4 (KL-type terms are sums of ~2e8 cancelling fp32 terms)
  student CE   rel 1e-5
  dlogits      stored bf16: per-element rel 1e-2 + 1e-3 x row max|g|; per-row abs sums rel 5e-3
"""
import json

import numpy as np
import pytest
import torch

from fixtures import HERE, VARIANT_OF, kd_fixture_names, kd_inputs, load_kd_fixture

pytestmark = pytest.mark.gpu


def _ops():
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops
    return ops


def _run(meta, t, s, labels, dev, kd_only=False):
    ops = _ops()
    tb = t.to(dev, torch.bfloat16)
    sb = s.to(dev, torch.bfloat16)
    lab = labels.to(dev)
    loss, dl = ops.kd_loss_fwd_bwd(
        sb, tb, lab, VARIANT_OF[meta["variant"]], temperature=meta["T"], alpha=meta["alpha"],
        kd_weight=meta["kd_weight"], ce_weight=0.0 if kd_only else meta["ce_weight"], check=True)
    torch.cuda.synchronize()
    return loss.cpu().double().numpy(), dl.float().cpu().reshape(-1, s.shape[-1])


def _close_rows(got, ref_rows, ref_idx, rtol=1e-2, frac=1e-3):
    for i, r in enumerate(ref_idx):
        ref = torch.from_numpy(ref_rows[i])
        g = got[int(r)]
        tol = rtol * ref.abs() + frac * ref.abs().max()
        bad = ((g - ref).abs() > tol).sum().item()
        assert bad == 0, f"row {r}: {bad} elements outside tolerance"


@pytest.mark.parametrize("name", kd_fixture_names())
def test_kd_loss_kernel_matches_reference(name, dev):
    meta, exp = load_kd_fixture(name)
    t, s, labels = kd_inputs(meta, exp)
    loss, g = _run(meta, t, s, labels, dev)
    assert loss[1] == pytest.approx(float(exp["ce"]), rel=1e-5)
    if meta["variant"] != "ce":  # BD SFT has no teacher (teacher CE side output absent)
        assert loss[2] == pytest.approx(float(exp["teacher_ce"]), rel=1e-5)
    assert loss[0] == pytest.approx(float(exp["kd_term"]), rel=1e-4, abs=1e-12)
    assert loss[3] == pytest.approx(float(exp["total"]), rel=1e-4)
    np.testing.assert_allclose(g.abs().sum(1).double().numpy(), exp["g_rowabs"], rtol=5e-3, atol=1e-12)
    _close_rows(g, exp["g_rows"], exp["g_rows_idx"])
    idx = exp["g_samp_idx"]
    ref = exp["g_samp_val"]
    got = g[idx[:, 0], idx[:, 1]].numpy()
    rowmax = np.abs(exp["g_rows"]).max()
    assert np.all(np.abs(got - ref) <= 1e-2 * np.abs(ref) + 1e-3 * rowmax)


@pytest.mark.parametrize("name", [n for n in kd_fixture_names() if not n.startswith("ce_")])
def test_kd_term_gradient_alone(name, dev):
    """The KD gradient is ~1e-6 of the CE's; check it in isolation (ce_weight = 0)."""
    meta, exp = load_kd_fixture(name)
    t, s, labels = kd_inputs(meta, exp)
    _, g = _run(meta, t, s, labels, dev, kd_only=True)
    np.testing.assert_allclose(g.abs().sum(1).double().numpy(), exp["gk_rowabs"], rtol=5e-3)
    _close_rows(g, exp["gk_rows"], exp["g_rows_idx"])
    idx = exp["g_samp_idx"]
    ref = exp["gk_samp_val"]
    got = g[idx[:, 0], idx[:, 1]].numpy()
    scale = np.abs(exp["gk_rows"]).max()
    assert np.all(np.abs(got - ref) <= 1e-2 * np.abs(ref) + 1e-3 * scale)


def test_loca_label_out_of_range_raises(dev):
    """KAT 2: a -100 label makes LoCa's gather raise in the reference; the kernel reports
    KD_ERR_LABEL_RANGE through kd_loss_check."""
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import _native as N
    ops = _ops()
    k = json.loads((HERE / "kat.json").read_text())["kat1"]
    V = 16
    t = torch.zeros(2, 5, 24, dtype=torch.bfloat16, device=dev)
    s = torch.zeros(2, 5, V, dtype=torch.bfloat16, device=dev)
    labels = torch.tensor(k["labels"], device=dev)
    labels[0, 0] = -100
    with pytest.raises(N.KdError) as e:
        ops.kd_loss_fwd_bwd(s, t, labels, "loca", check=True)
    assert e.value.code == 5


def test_kat1_small_vocab_against_reference(dev):
    """KAT 1 inputs (V=16, duplicate labels) through the kernel, padded to V % 8 == 0."""
    ops = _ops()
    k = json.loads((HERE / "kat.json").read_text())["kat1"]
    t = torch.tensor(k["t"])  # [2, 5, 19]
    s = torch.tensor(k["s"])  # [2, 5, 16]
    tt = torch.full((2, 5, 24), -30.0)
    tt[..., :19] = t
    # bf16 rounding of these fp32 inputs changes the loss at the 1e-3 level; compare with
    # the oracle on the same bf16-rounded values instead, and with the reference loosely
    from oracle import kd_losses as O
    tb, sb = tt.bfloat16(), s.bfloat16()
    loss, dl = ops.kd_loss_fwd_bwd(sb.to(dev), tb.to(dev), torch.tensor(k["labels"]).to(dev), "loca",
                                   temperature=1.0, kd_weight=1.0, ce_weight=0.0, check=True)
    ref = O.loca_kd_term(tb.float()[..., :19], sb.float(), torch.tensor(k["labels"]), T=1.0)
    assert float(loss[0]) == pytest.approx(ref.item(), rel=1e-5)
    assert float(loss[0]) == pytest.approx(k["loss"], rel=5e-2)
