"""End-to-end parity report: every per-term value of the HIP training_step vs the
reference's own forward (tests/golden/model_*.npz), as measured deltas.

    python tools/parity_report.py [--out profiles/r02/parity.json]

For each module kind: KD term, student CE, teacher CE, NT-Xent, total (|Δ|, rel Δ and
whether |Δ| <= 1e-4 + 1e-3 |ref|, the north-star tolerance); student logits per-row
logsumexp and sampled rows; the student gradient's total norm.  GPU only.
"""
from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "tests" / "golden"))

ATOL, RTOL = 1e-4, 1e-3


def _d(got, ref):
    ad = abs(got - ref)
    return dict(got=got, ref=ref, abs=ad, rel=ad / abs(ref) if ref else None, ok=bool(ad <= ATOL + RTOL * abs(ref)))


def measure(name, dev):
    import numpy as np
    import torch
    from model_fixtures import ALL_KINDS, batch, load
    from test_kd_step_gpu import _module
    meta, exp = load(name)
    kind, phase = ALL_KINDS[name]
    m = _module(kind, phase)
    m.keep_logits = True
    b = batch(meta, dev)
    loss = m.training_step(b, 0)
    loss.backward()
    torch.cuda.synchronize()
    kd, ce, tce, tot = m.last_terms.tolist()
    out = {"total": _d(loss.item(), float(exp["total"])), "student_ce": _d(ce, float(exp["student_ce"]))}
    if not math.isnan(float(exp["teacher_ce"])):
        out["teacher_ce"] = _d(tce, float(exp["teacher_ce"]))
    if not math.isnan(float(exp["kd_term"])):
        out["kd_term"] = _d(kd, float(exp["kd_term"]))
    if not math.isnan(float(exp["ntxent"])):
        out["ntxent"] = _d(float(m.last_ntxent[1]), float(exp["ntxent"]))
    s3, _ = m.last_logits
    lse = torch.logsumexp(s3.double(), -1).reshape(-1).cpu().numpy()
    dl = np.abs(lse - exp["s_logit_lse"])
    out["s_logit_lse"] = dict(max_abs=float(dl.max()), max_rel=float((dl / np.abs(exp["s_logit_lse"])).max()),
                              ok=bool((dl <= ATOL + RTOL * np.abs(exp["s_logit_lse"])).all()))
    rows = exp["logit_rows"].tolist()
    st = int(exp["logit_col_stride"])
    got = s3[:, rows, ::st].float().cpu().numpy()
    ref = exp["s_logit_rows"]
    err = np.abs(got - ref)
    out["s_logit_rows"] = dict(max_abs=float(err.max()), rms_ref=float(np.sqrt((ref ** 2).mean())),
                               max_rel_to_rms=float(err.max() / np.sqrt((ref ** 2).mean())),
                               frac_within_north_star=float((err <= ATOL + RTOL * np.abs(ref)).mean()))
    P = m.student_model.P
    names = [str(n) for n in exp["grad_names"]]
    hip = {}
    for n in names:
        g = P.grad_view(n)
        spec = next(s for s in P.specs if s.name == n)
        if spec.ckpt_shape is not None:
            g = g[:, :int(np.prod(spec.ckpt_shape[1:]))]
        hip[n] = g.double().cpu().reshape(-1)
    tot2 = sum(float(g.pow(2).sum()) for g in hip.values())
    out["grad_total_norm"] = _d(math.sqrt(tot2), float(exp["grad_total_norm"]))
    # the yardstick: the same oracle (pinned fp32 restatement) run in bf16 on the CPU
    from model_fixtures import grad_total_norm, oracle_grads
    _, bgr, blog = oracle_grads(name, torch.bfloat16, with_logits=True)
    out["grad_total_norm"]["bf16_oracle"] = _d(grad_total_norm(bgr), float(exp["grad_total_norm"]))
    berr = np.abs(blog[:, rows, ::st].float().numpy() - ref)
    out["s_logit_rows"]["bf16_oracle_frac_within_north_star"] = float((berr <= ATOL + RTOL * np.abs(ref)).mean())
    out["s_logit_rows"]["bf16_oracle_max_abs"] = float(berr.max())
    # per parameter group: where the total-norm difference comes from
    _, fgr = oracle_grads(name)
    out["grad_groups"] = groups(hip, {k: v.double().reshape(-1) for k, v in fgr.items()},
                                {k: v.double().reshape(-1) for k, v in bgr.items()})
    return out


def _group(name: str) -> str:
    for tag in ("embed_tokens", "lm_head", "model.norm.weight", "patch_embedding", "position_embedding",
                "post_layernorm", "multi_modal_projector", "image_newline"):
        if tag in name:
            return name
    return ".".join(p for p in name.split(".") if not p.isdigit())


def groups(hip, f32, b16):
    """{group: rel norm delta of HIP and of the bf16 oracle vs fp32, and each one's share of
    the total squared-norm difference, and |HIP - fp32| / |fp32|}."""
    acc = {}
    for n, g in hip.items():
        r = acc.setdefault(_group(n), [0.0, 0.0, 0.0, 0.0])
        r[0] += float(f32[n].pow(2).sum()); r[1] += float(g.pow(2).sum()); r[2] += float(b16[n].pow(2).sum())
        r[3] += float((g - f32[n]).pow(2).sum())
    t = [sum(r[i] for r in acc.values()) for i in range(3)]
    res = {}
    for k, (a, h, b, d) in sorted(acc.items(), key=lambda kv: -abs(kv[1][1] - kv[1][0])):
        if a == 0:
            continue
        res[k] = dict(norm=math.sqrt(a), hip_rel=math.sqrt(h / a) - 1, bf16_oracle_rel=math.sqrt(b / a) - 1,
                      hip_share=(h - a) / (t[1] - t[0]) if t[1] != t[0] else None,
                      hip_err_rel=math.sqrt(d / a))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("kinds", nargs="*")
    a = ap.parse_args()
    import torch
    from model_fixtures import KINDS
    dev = torch.device("cuda:0")
    rep = {"tolerance": f"|d| <= {ATOL} + {RTOL} |ref| (north_star)"}
    for name in (a.kinds or KINDS):
        rep[name] = measure(name, dev)
        print(name, json.dumps(rep[name]), flush=True)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
