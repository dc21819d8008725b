"""Shared measurement of one HIP training_step against an end-to-end fixture
(tests/golden/model_*.npz): the loss terms, the student logits, and every parameter's
gradient against the reference's, each next to the bf16 floor (the pinned oracle run in
plain bf16, tests/golden/bf16_floor.json).  Used by tests/test_kd_step_gpu.py and
tools/parity_report.py.  GPU only.

Per-parameter gradient bound (every parameter the reference differentiates), never looser than
1 % on the norm and 0.99 on the cosine:
  norm   | |g| / |g_ref| - 1 |  <=  min(1e-2, max(1e-3, 1.5 x the bf16 floor's own norm miss,
                                      0.25 x the bf16 floor's relative error |g_bf16 - g_ref| / |g_ref|))
  cosine cos(g, g_ref)        >=  max(0.99, the bf16 floor's cosine - 1e-3)
The floor's relative error is sqrt(2 (1 - cos_floor)); a quarter of it covers parameters whose
gradient is so small that bf16 noise decides its norm (the Qwen2 k_proj.bias, ~1e-6 of the
largest gradient: HIP 0.29 % vs the floor's 0.18 % norm miss, both at cosine 0.99996+).
Where the bf16 floor itself is noise (floor cosine < 0.99 or floor norm miss > 5 %: gradients that
are a cancelling sum, e.g. the NT-Xent-only SigLIP post_layernorm.bias, whose two tiles'
contributions cancel to ~8e-4 of each, tools/ntx_bias_study.py) a parameter outside that bound may
instead meet an ABSOLUTE one:  |g - g_ref| <= 1e-3 x |the same layer's weight gradient (reference)|.
g_ref: the fp32 oracle's full gradient for the tiny fixtures (the oracle is pinned to the
reference's recorded norms and heads, tests/test_oracle_model.py); the reference's own
gradient at GRAD_SAMPLE seeded positions for the real-width fixtures; |g_ref| is always the
reference's own recorded norm.

Exception: the SigLIP key-projection biases (`vision_tower...self_attn.k_proj.bias`) have an
exactly zero gradient: q . b_k is the same for every key of a query, and softmax is invariant
to a per-row shift (the reference records fp32 noise, 1e-13..1e-10 of the largest parameter
gradient, with cosines near 0 between runs).  For them the bound is |g| <= ZERO_REL x the
reference norm of the same layer's q_proj.bias gradient (HIP: 2.5e-5 .. 8.8e-4 of it,
profiles/r04/parity.json; a key-bias gradient that failed to cancel would be of its order).
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import numpy as np
import torch

from model_fixtures import EVERY_KIND, batch, grad_sample_index, load, module_names, oracle_grads

ATOL, RTOL = 1e-4, 1e-3   # north_star
FLOOR = json.loads((Path(__file__).resolve().parent / "golden" / "bf16_floor.json").read_text())
NORM_MIN, NORM_FLOOR_X, FLOOR_ERR_X, COS_SLACK = 1e-3, 1.5, 0.25, 1e-3
NORM_CAP, COS_CAP = 1e-2, 0.99          # no bound looser than 1 % on the norm / 0.99 on the cosine
NOISE_NORM, ABS_REL = 0.05, 1e-3        # the bf16 floor is noise: absolute criterion vs the layer's weight
ZERO_REL = 1e-2


def exactly_zero(name: str) -> bool:
    """Parameters whose gradient vanishes in exact arithmetic (see the module docstring)."""
    return name.startswith("vision_tower.") and name.endswith("self_attn.k_proj.bias")

_WEIGHTS = {}   # model name -> flat bf16 weights (the real-width models' CPU-RNG init is slow)


def module(kind, phase, names=("tiny-student", "tiny-teacher")):
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
    sn, tn = names
    cached = sn in _WEIGHTS and (kind == "bd" or tn in _WEIGHTS)
    kw = dict(seed_student=None, seed_teacher=None) if cached else {}
    if kind == "lb":
        m = K.LogitBasedKD(sn, tn, **kw)
    elif kind == "dt":
        m = K.OnlineKnowledgeDistillationLLavaOneVision(sn, tn, phase=phase, **kw)
        if phase == 1:
            m.freeze_student_language_layers()
        if phase == 2:
            m.freeze_student_vision_layers()
    elif kind == "fb":
        m = K.FeatureBasedKD(sn, tn, **kw)
    else:
        m = K.LlavaOnevisionModule(sn, **kw)
    if sn.startswith("real"):
        if cached:
            m.student_model.P.flat.copy_(_WEIGHTS[sn])
            m.student_model.P.master.copy_(_WEIGHTS[sn].float())
            if m.teacher_model is not None:
                m.teacher_model.P.flat.copy_(_WEIGHTS[tn])
        else:
            _WEIGHTS[sn] = m.student_model.P.flat.clone()
            if m.teacher_model is not None:
                _WEIGHTS[tn] = m.teacher_model.P.flat.clone()
    return m


def hip_grad(P, name):
    """The HIP gradient of `name` in the reference's shape (the conv weight's pad columns dropped)."""
    g = P.grad_view(name)
    spec = next(s for s in P.specs if s.name == name)
    if spec.ckpt_shape is not None:
        g = g[:, :math.prod(spec.ckpt_shape[1:])]
    return g


def run_step(name, dev):
    """One training_step + backward of the drop-in module on the fixture's batch."""
    meta, exp = load(name)
    kind, phase = EVERY_KIND[name]
    m = module(kind, phase, module_names(meta))
    m.keep_logits = True
    loss = m.training_step(batch(meta, dev), 0)
    assert loss.requires_grad and loss.dim() == 0
    loss.backward()
    torch.cuda.synchronize()
    return m, meta, exp, loss


def logit_report(m, exp):
    s3, _ = m.last_logits
    lse = torch.logsumexp(s3.double(), -1).reshape(-1).cpu().numpy()
    ref_lse = exp["s_logit_lse"]
    dl = np.abs(lse - ref_lse)
    got = s3[:, exp["logit_rows"].tolist(), ::int(exp["logit_col_stride"])].float().cpu().numpy()
    ref = exp["s_logit_rows"]
    err = np.abs(got - ref)
    return dict(lse_max_abs=float(dl.max()), lse_max_rel=float((dl / np.abs(ref_lse)).max()),
                lse_ok=bool((dl <= ATOL + RTOL * np.abs(ref_lse)).all()),
                rows_frac_within_north_star=float((err <= ATOL + RTOL * np.abs(ref)).mean()),
                rows_max_abs=float(err.max()))


def param_report(name, m, exp):
    """{parameter: norm_rel, cos, the floor's, the bounds, ok} for every parameter the
    reference differentiates, plus the gradient's total norm."""
    P = m.student_model.P
    names = [str(n) for n in exp["grad_names"]]
    fl = FLOOR[name]["params"]
    real = "grad_samples" in exp
    ref32 = None if real else oracle_grads(name)[1]
    rep, tot = {}, 0.0
    ref_norm = {n: float(v) for n, v in zip(names, exp["grad_norms"])}
    for i, n in enumerate(names):
        g = hip_grad(P, n).double().cpu().reshape(-1)
        tot += float(g.pow(2).sum())
        rn = float(exp["grad_norms"][i])
        if real:
            idx = grad_sample_index(n, g.numel())
            a, b = g[idx], torch.from_numpy(exp["grad_samples"][i][:idx.numel()]).double()
        else:
            a, b = g, ref32[n].double().reshape(-1)
        cos = float((a @ b) / (a.norm() * b.norm() + 1e-300))
        norm_rel = abs(float(g.norm()) / rn - 1) if rn > 0 else float(g.norm())
        f = fl[n]
        if exactly_zero(n):
            gz = float(g.norm())
            qn = ref_norm[n.replace("k_proj.bias", "q_proj.bias")]
            rep[n] = dict(ref_norm=rn, norm=gz, q_bias_ref_norm=qn, ratio=gz / qn, bound_ratio=ZERO_REL,
                          exactly_zero=True, ok=bool(gz <= ZERO_REL * qn))
            continue
        bn = min(NORM_CAP, max(NORM_MIN, NORM_FLOOR_X * f["norm_rel"],
                               FLOOR_ERR_X * math.sqrt(max(0.0, 2 * (1 - f["cos"])))))
        bc = max(COS_CAP, f["cos"] - COS_SLACK)
        r = dict(ref_norm=rn, norm_rel=norm_rel, cos=cos, floor_norm_rel=f["norm_rel"], floor_cos=f["cos"],
                 bound_norm_rel=bn, bound_cos=bc, ok=bool(norm_rel <= bn and cos >= bc), criterion="relative")
        noise = f["cos"] < COS_CAP or f["norm_rel"] > NOISE_NORM
        wname = n[:-len("bias")] + "weight" if n.endswith(".bias") else None
        if not r["ok"] and noise and wname in ref_norm:
            # |g - g_ref| over the compared entries, scaled to the whole tensor when they are a sample
            err = float((a - b).norm()) * math.sqrt(g.numel() / a.numel())
            bound = ABS_REL * ref_norm[wname]
            r.update(abs_err=err, abs_bound=bound, weight_ref_norm=ref_norm[wname], ok=bool(err <= bound),
                     criterion="absolute (bf16 floor is noise)")
        rep[n] = r
    ref_gn = float(exp["grad_total_norm"])
    gn = math.sqrt(tot)
    return rep, dict(got=gn, ref=ref_gn, rel=(gn - ref_gn) / ref_gn,
                     floor_rel=(FLOOR[name]["grad_total_norm"] - ref_gn) / ref_gn)
