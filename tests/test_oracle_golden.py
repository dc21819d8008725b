"""The CPU oracle (oracle/kd_losses.py) against outputs recorded from the reference.

Fixtures were produced by tests/golden/make_golden.py running the reference's own
compute_loca_loss / compute_vision_loss / compute_loss / contrastive_loss (and
transformers' ForCausalLMLoss) in this container.  CPU only.
"""
import json

import numpy as np
import pytest
import torch

from oracle import kd_losses as O
from fixtures import HERE, kd_fixture_names, kd_inputs, load_kd_fixture

KAT = json.loads((HERE / "kat.json").read_text())


def test_kat1_loca_global_last_write_wins():
    k = KAT["kat1"]
    t = torch.tensor(k["t"]); s = torch.tensor(k["s"], requires_grad=True)
    labels = torch.tensor(k["labels"])
    loss = O.loca_kd_term(t, s, labels, T=k["T"], alpha=0.8)
    loss.backward()
    assert loss.item() == pytest.approx(k["loss"], rel=1e-6)
    np.testing.assert_allclose(s.grad.numpy(), np.array(k["grad"]), rtol=1e-5, atol=1e-9)
    # the calibrated-teacher matrix: every row carries the same override columns
    q_ref = np.array(k["q"])
    V = s.shape[-1]
    p_t = O._softmax_T(t[..., :V], k["T"])
    lab_last = O.last_position_table(labels.numpy(), V)
    for v in range(V):
        col = q_ref[..., v]
        if lab_last[v] >= 0 or (O.last_position_table(O.top2_second_index(p_t).numpy(), V)[v] >= 0):
            assert np.allclose(col, col.reshape(-1)[0]), f"column {v} should be row-independent"
        else:
            np.testing.assert_allclose(col, p_t[..., v].numpy(), rtol=1e-6)


def test_kat2_label_minus100_raises():
    assert KAT["kat2"]["raised"] and KAT["kat2"]["type"] == "RuntimeError"
    k = KAT["kat1"]
    t = torch.tensor(k["t"]); s = torch.tensor(k["s"])
    labels = torch.tensor(k["labels"]); labels[0, 0] = -100
    with pytest.raises(RuntimeError):
        O.loca_kd_term(t, s, labels, T=1.0)


def test_kat5_clamp_zeroes_gradient():
    k = KAT["kat5"]
    t = torch.tensor(k["t"]); s = torch.tensor(k["s"], requires_grad=True)
    loss = O.loca_kd_term(t, s, torch.tensor(k["labels"]), T=1.0)
    loss.backward()
    assert loss.item() == pytest.approx(k["loss"], rel=1e-6)
    np.testing.assert_allclose(s.grad.numpy(), np.array(k["grad"]), rtol=1e-5, atol=1e-12)


def test_kat6_topk_tie_order_documented():
    # torch CPU topk(2) on [.1,.5,.3,.5,.5,.2] returns [1,4]; the oracle/kernel pick
    # the lowest index on ties (-> second = 3).  Fixtures are constructed tie-free.
    assert KAT["kat6"]["topk2_indices"] == [[1, 4]]
    assert O.top2_second_index(torch.tensor(KAT["kat6"]["values"])).tolist() == [3]


def test_kat9_image_token_counts_recorded():
    assert KAT["kat9"]["336x336"] == {"num_patches": 2, "num_tokens": 1485}
    assert KAT["kat9"]["480x640"] == {"num_patches": 5, "num_tokens": 2929}


def test_ntxent_matches_reference():
    import inputs as I
    k = KAT["ntxent"]
    sf, tf = I.features(k["n"], k["dim"], seed=k["seed"], tokens=k["tokens"])
    assert np.allclose(I.checksum(sf), k["s_ck"], rtol=1e-12)
    sf.requires_grad_(True)
    loss = O.nt_xent(O.pooled_features(sf), O.pooled_features(tf))
    loss.backward()
    # loss = lse - diag with both ~ 1/0.07 = 14.3 in fp32: absolute floor ~ 1 ulp(14.3) ~ 1e-6
    assert loss.item() == pytest.approx(k["loss"], abs=2e-6)
    g = sf.grad.double()
    assert float(g.abs().sum()) == pytest.approx(k["grad_abs"], rel=1e-4)
    np.testing.assert_allclose(sf.grad[0, 0, :16].numpy(), np.array(k["grad_row0"]), rtol=1e-4, atol=1e-12)


@pytest.mark.parametrize("name", kd_fixture_names())
def test_oracle_kd_losses_match_reference(name):
    meta, exp = load_kd_fixture(name)
    t, s, labels = kd_inputs(meta, exp)
    s.requires_grad_(True)
    var, T = meta["variant"], meta["T"]
    ce = O.causal_lm_ce(s, labels)
    if var == "loca":
        kd = O.loca_kd_term(t, s, labels, T=T, alpha=meta["alpha"])
    elif var == "kl":
        kd = O.kl_mean_term(t, s, T)
    elif var == "kllt":
        kd = O.kl_logtarget_term(t, s, T)
    else:
        kd = torch.zeros(())
    total = meta["kd_weight"] * kd + meta["ce_weight"] * ce
    assert ce.item() == pytest.approx(float(exp["ce"]), rel=2e-6)
    assert kd.item() == pytest.approx(float(exp["kd_term"]), rel=2e-5, abs=1e-12)
    assert total.item() == pytest.approx(float(exp["total"]), rel=2e-5)
    with torch.no_grad():
        tce = O.causal_lm_ce(t, labels)
    assert tce.item() == pytest.approx(float(exp["teacher_ce"]), rel=2e-6)
    total.backward()
    V = s.shape[-1]
    g = s.grad.reshape(-1, V)
    np.testing.assert_allclose(g.abs().sum(1).double().numpy(), exp["g_rowabs"], rtol=1e-4)
    idx = exp["g_samp_idx"]
    np.testing.assert_allclose(g[idx[:, 0], idx[:, 1]].numpy(), exp["g_samp_val"], rtol=1e-4, atol=1e-13)


@pytest.mark.parametrize("name", [n for n in kd_fixture_names() if "loca" in n][:3])
def test_chunked_loca_matches_reference(name):
    """oracle.loca_kd_term_rows (row chunks, any device; the c4 fp8 KD-term split in bench.py /
    tests/test_fp8_gpu.py) gives the reference's compute_loca_loss KD term; with its own second
    index passed explicitly, the same value."""
    meta, exp = load_kd_fixture(name)
    t, s, labels = kd_inputs(meta, exp)
    kd = O.loca_kd_term_rows(t, s, labels, T=meta["T"], alpha=meta["alpha"], rows_per_chunk=97)
    assert kd == pytest.approx(float(exp["kd_term"]), rel=2e-5, abs=1e-12)
    V = s.shape[-1]
    k = O.top2_second_index(O._softmax_T(t[..., :V], meta["T"]))
    assert O.loca_kd_term_rows(t, s, labels, T=meta["T"], alpha=meta["alpha"], k=k) == pytest.approx(kd, rel=1e-6)


def test_chunked_loca_kat1():
    k = KAT["kat1"]
    kd = O.loca_kd_term_rows(torch.tensor(k["t"]), torch.tensor(k["s"]), torch.tensor(k["labels"]), T=k["T"],
                             rows_per_chunk=1)
    assert kd == pytest.approx(k["loss"], rel=1e-6)
