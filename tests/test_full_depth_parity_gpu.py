"""BASELINE config c1 at FULL depth against the pinned fp32 oracle on the same weights
(tests/full_depth.py): the logit-based KD step (LB:125-169, compute_loca_loss at T = 1,
LB:208-261) with the real 7B teacher (SigLIP 26 layers, Qwen2-7B 28) and 0.5B student (26 +
24), L = 1536, one 336x336 sample; the reference's LB teacher and student are fp32 end to end
(LB:29-33), and so is the oracle here.

Held (north_star: |d| <= 1e-4 + 1e-3 |ref|; measured on MI355X, profiles/r05/full_depth.json):
  KD term, student CE, teacher CE, total         north_star        (2.2e-5 / 1.1e-5 / 1.0e-4 / 1.1e-5 rel)
  per-row logsumexp, student and teacher logits  north_star, every row   (max 9.8e-6 / 7.2e-5 rel)
  gradient total norm                            rel <= 1e-3       (-1.5e-4)
  every parameter's gradient                     norm within 1 %, cosine >= 0.999 vs the oracle's
                                                 full fp32 gradient (worst: 0.85 % / 0.99972)
  SigLIP k_proj.bias (exactly zero in exact arithmetic, tests/step_parity.py)
                                                 |g| <= 1e-2 |q_proj.bias grad| of the same layer
  raw student logits (48 sampled rows x 151,936) fraction within north_star >= 0.10 (0.119; plain
                                                 bf16 oracle 0.044): the bf16 rounding of the
                                                 lm_head INPUT alone leaves 0.41 (stated, not held)
"""
import pytest
import torch

from full_depth import compare, hip_step, oracle_step

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(1200)
def test_c1_full_depth_matches_fp32_oracle(dev):
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    hip, tsd, ssd = hip_step(dev)
    ref = oracle_step(tsd, ssd, torch.float32)
    r = compare(hip, ref, ssd["language_model.model.embed_tokens.weight"])
    del tsd, ssd
    for k, v in r["terms"].items():
        assert v["ok"], (k, v)
    assert r["s_lse"]["ok"], r["s_lse"]
    assert r["t_lse"]["ok"], r["t_lse"]
    assert r["grad_total_norm"]["ok"], r["grad_total_norm"]
    per = r["grad_params"]
    for n, v in per.items():
        if n.startswith("vision_tower.") and n.endswith("self_attn.k_proj.bias"):
            qn = float(hip["grads"][n.replace("k_proj.bias", "q_proj.bias")].double().norm())
            gz = float(hip["grads"][n].double().norm())
            assert gz <= 1e-2 * qn, (n, gz, qn)
            continue
        assert abs(v["norm_rel"]) <= 1e-2 and v["cos"] >= 0.999, (n, v)
    assert r["s_logits_rows"]["frac_within"] >= 0.10, r["s_logits_rows"]
    # the KD target itself: the teacher's raw logits (bf16 Qwen2-7B residual stream; the reference's
    # LB teacher runs fp32, LB:29-33) within 4 % rel-L2 of the fp32 teacher (measured 3.1 %; with
    # teacher_residual_f32=True 2.3 %, profiles/r05/full_depth.json), every row's lse at north_star
    assert r["t_logits_rows"]["rel_l2"] <= 0.04, r["t_logits_rows"]
    # the fp32-output lm_head on the same hidden state: the bf16 rounding of the stored logits
    # is not where the raw-logit misses come from
    assert r["s_logits_rows_f32_out"]["frac_within"] >= r["s_logits_rows"]["frac_within"] - 0.01


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["dt1", "dt2", "dt3", "fb", "bd"])
def test_every_module_full_depth_matches_fp32_oracle(name, dev):
    """The other modules at FULL depth against the pinned fp32 oracle on the same weights
    (tests/full_depth.py measure_kinds; profiles/r05/full_depth_kinds.json): the double-trouble
    phases 1-3 (DT:250-260; phase 1 LM frozen, phase 2 ViT frozen), FeatureBasedKD (FB:161-165,
    NT-Xent on the post-LN features) and the depth-student SFT baseline (BD:90-101), bs 1, L 1536.
    Held: the total at north_star, every row's student logsumexp at north_star, the gradient total
    norm within 1e-3, every trainable parameter's gradient within 1 % norm / cosine 0.999 except
    the SigLIP k_proj.bias (exactly zero in exact arithmetic, tests/step_parity.py).
    Measured: totals rel <= 4.1e-5, gradient norms rel <= 3.0e-4, worst other parameter cos 0.9997."""
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    from full_depth import measure_kinds
    r = measure_kinds(dev, [name])[name]
    for k, v in r["terms"].items():
        assert v["ok"], (k, v)
    assert r["s_lse"]["ok"], r["s_lse"]
    assert r["grad_total_norm"]["ok"], r["grad_total_norm"]
    for n, v in r["grad_params"].items():
        if n.startswith("vision_tower.") and n.endswith("self_attn.k_proj.bias"):
            # |g| (both ~0: softmax is invariant to a key bias) within 1e-2 of the layer's q_proj.bias gradient
            gz = (v["norm_rel"] + 1.0) * v["ref_norm"] if v["ref_norm"] > 0 else v["norm_rel"]
            qn = r["grad_params"][n.replace("k_proj.bias", "q_proj.bias")]["ref_norm"]
            assert gz <= 1e-2 * qn, (n, gz, qn)
            continue
        assert abs(v["norm_rel"]) <= 1e-2 and v["cos"] >= 0.999, (n, v)


@pytest.mark.timeout(900)
def test_c4_full_depth_matches_fp32_oracle(dev):
    """BASELINE config c4's own configuration at FULL depth (tests/full_depth.py measure_c4): the
    double-trouble phase 3 module (DT:257-260, LoCa at T = 0.8, DT:141-194) with the fp8 (e4m3,
    lm_mlp) teacher, bs 1, against the pinned fp32 oracle running the fp32 teacher on the same
    weights.  Held: student CE, total, every student lse row and the gradient total norm at
    north_star (the student side never sees the teacher's precision except through the LoCa
    target); the KD term and the teacher CE within the fp8 teacher's stated 1 %; every trainable
    parameter's gradient within 1 % norm / cosine 0.999 (SigLIP k_proj.bias as above)."""
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    from full_depth import C4_FP8_TOL, measure_c4
    r = measure_c4(dev)
    t = r["terms"]
    for k in ("student_ce", "total"):
        assert t[k]["ok"], (k, t[k])
    for k in ("kd_term", "teacher_ce"):
        assert t[k]["rel"] <= C4_FP8_TOL, (k, t[k])
    assert r["s_lse"]["ok"], r["s_lse"]
    assert r["grad_total_norm"]["ok"], r["grad_total_norm"]
    for n, v in r["grad_params"].items():
        if n.startswith("vision_tower.") and n.endswith("self_attn.k_proj.bias"):
            gz = (v["norm_rel"] + 1.0) * v["ref_norm"] if v["ref_norm"] > 0 else v["norm_rel"]
            qn = r["grad_params"][n.replace("k_proj.bias", "q_proj.bias")]["ref_norm"]
            assert gz <= 1e-2 * qn, (n, gz, qn)
            continue
        assert abs(v["norm_rel"]) <= 1e-2 and v["cos"] >= 0.999, (n, v)


@pytest.mark.timeout(1200)
def test_sunrgbd_geometry_full_depth_matches_fp32_oracle(dev):
    """c1's module (LB, LoCa T = 1) at FULL depth on a real SUNRGBD image size: 480x640 -> anyres
    5 tiles (base + 2x2 grid), 2,929 image tokens with the unpadded grid's newlines, L = 2,980 (SURVEY
    KAT 9, DM:124-146, DS:185-212), bs 1, against the fp32 oracle on the same weights.  Held as the
    336x336 case: every term, every student and teacher lse row at north_star, the gradient total norm
    within 1e-3, every parameter within 1 % norm / cosine 0.999 (SigLIP k_proj.bias as above)."""
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    from full_depth import geometry
    with geometry((480, 640)):
        hip, tsd, ssd = hip_step(dev)
        ref = oracle_step(tsd, ssd, torch.float32)
        r = compare(hip, ref, None)
    del tsd, ssd
    for k, v in r["terms"].items():
        assert v["ok"], (k, v)
    assert r["s_lse"]["ok"], r["s_lse"]
    assert r["t_lse"]["ok"], r["t_lse"]
    assert r["grad_total_norm"]["ok"], r["grad_total_norm"]
    for n, v in r["grad_params"].items():
        if n.startswith("vision_tower.") and n.endswith("self_attn.k_proj.bias"):
            qn = float(hip["grads"][n.replace("k_proj.bias", "q_proj.bias")].double().norm())
            gz = float(hip["grads"][n].double().norm())
            assert gz <= 1e-2 * qn, (n, gz, qn)
            continue
        assert abs(v["norm_rel"]) <= 1e-2 and v["cos"] >= 0.999, (n, v)
