"""End-to-end parity report: every per-term value of the HIP training_step vs the
reference's own forward (tests/golden/model_*.npz), as measured deltas.

    python tools/parity_report.py [--out profiles/r02/parity.json]

For each module kind: KD term, student CE, teacher CE, NT-Xent, total (|Δ|, rel Δ and
whether |Δ| <= 1e-4 + 1e-3 |ref|, the north-star tolerance); student logits per-row
logsumexp and sampled rows; the student gradient's total norm and every parameter's norm /
cosine against the reference next to the bf16 floor (tests/step_parity.py).  GPU only.
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
    from step_parity import logit_report, param_report, run_step
    m, meta, exp, loss = run_step(name, dev)
    kd, ce, tce, tot = m.last_terms.tolist()
    out = {"total": _d(loss.item(), float(exp["total"])), "student_ce": _d(ce, float(exp["student_ce"]))}
    if not math.isnan(float(exp["teacher_ce"])):
        out["teacher_ce"] = _d(tce, float(exp["teacher_ce"]))
    if not math.isnan(float(exp["kd_term"])):
        out["kd_term"] = _d(kd, float(exp["kd_term"]))
    if not math.isnan(float(exp["ntxent"])):
        out["ntxent"] = _d(float(m.last_ntxent[1]), float(exp["ntxent"]))
    from step_parity import FLOOR
    fl = FLOOR[name]
    lr = logit_report(m, exp)
    lr.update(bf16_floor_frac_within_north_star=fl["logit_frac_within_north_star"],
              bf16_floor_max_abs=fl["logit_max_abs"])
    out["s_logits"] = lr
    m.last_logits = None
    per, totn = param_report(name, m, exp)
    out["grad_total_norm"] = totn
    out["grad_params"] = per
    out["grad_params_ok"] = f"{sum(r['ok'] for r in per.values())}/{len(per)}"
    # per parameter group: where the total-norm difference comes from (tiny fixtures: full vectors)
    if "grad_samples" not in exp:
        from model_fixtures import oracle_grads
        from step_parity import hip_grad
        P = m.student_model.P
        hip = {str(n): hip_grad(P, str(n)).double().cpu().reshape(-1) for n in exp["grad_names"]}
        _, bgr = oracle_grads(name, torch.bfloat16)
        _, fgr = oracle_grads(name)
        out["grad_groups"] = groups(hip, {k: v.double().reshape(-1) for k, v in fgr.items()},
                                    {k: v.double().reshape(-1) for k, v in bgr.items()})
    del m
    torch.cuda.empty_cache()
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
    ap.add_argument("--full-depth", action="store_true",
                    help="c1 at full depth vs the fp32 oracle on the same weights (tests/full_depth.py)")
    ap.add_argument("--floor", action="store_true", help="--full-depth: also the plain-bf16 oracle (the floor)")
    ap.add_argument("--teacher-stream-ab", action="store_true",
                    help="--full-depth: also the HIP step with the teacher's Qwen2 residual stream in fp32")
    ap.add_argument("--teacher-fp8", default=None, metavar="POLICY",
                    help="--full-depth: also the HIP step with the fp8 (e4m3) teacher of c4 (e.g. lm_mlp)")
    ap.add_argument("--full-depth-kinds", nargs="+", default=None, metavar="KIND",
                    help="each module kind (tests/full_depth.KINDS: lb dt1 dt2 dt3 fb bd) at full depth vs the fp32 oracle")
    ap.add_argument("--c4-full-depth", action="store_true",
                    help="BASELINE c4 itself at full depth: DT phase 3 + the fp8 lm_mlp teacher vs the fp32 oracle")
    ap.add_argument("--image", default=None, metavar="HxW",
                    help="--full-depth on this image size (e.g. 480x640: SUNRGBD geometry, 5 tiles, L 2980)")
    ap.add_argument("--depth-profile", action="store_true",
                    help="the student's hidden-state error vs the fp32 oracle along both towers (tests/full_depth.py)")
    ap.add_argument("kinds", nargs="*")
    a = ap.parse_args()
    import torch
    if a.depth_profile:
        from full_depth import measure_depth_profile
        rep = measure_depth_profile(torch.device("cuda:0"))
        print(json.dumps(rep, indent=1), flush=True)
        if a.out:
            Path(a.out).parent.mkdir(parents=True, exist_ok=True)
            Path(a.out).write_text(json.dumps(rep, indent=1))
        return
    if a.c4_full_depth:
        from full_depth import measure_c4
        rep = measure_c4(torch.device("cuda:0"))
        print("c4", json.dumps({k: v for k, v in rep.items() if k != "grad_params"})[:3000], flush=True)
        if a.out:
            Path(a.out).parent.mkdir(parents=True, exist_ok=True)
            Path(a.out).write_text(json.dumps(rep, indent=1))
        return
    if a.full_depth_kinds:
        from full_depth import measure_kinds
        rep = measure_kinds(torch.device("cuda:0"), a.full_depth_kinds)
        for k in a.full_depth_kinds:
            r = {kk: vv for kk, vv in rep[k].items() if kk != "grad_params"}
            print(k, json.dumps(r)[:1500], flush=True)
        if a.out:
            Path(a.out).parent.mkdir(parents=True, exist_ok=True)
            Path(a.out).write_text(json.dumps(rep, indent=1))
        return
    if a.full_depth:
        from full_depth import geometry, measure as fd_measure
        hw = tuple(int(v) for v in a.image.split("x")) if a.image else (336, 336)
        with geometry(hw):
            rep = fd_measure(torch.device("cuda:0"), floor=a.floor, teacher_stream_ab=a.teacher_stream_ab,
                             teacher_fp8=a.teacher_fp8)
        rep["image"] = list(hw)
        for k in ("hip", "hip_teacher_stream_f32", "hip_teacher_fp8", "bf16_floor"):
            if k in rep:
                r = {kk: vv for kk, vv in rep[k].items() if kk != "grad_params"}
                print(k, json.dumps(r), flush=True)
        if a.out:
            Path(a.out).parent.mkdir(parents=True, exist_ok=True)
            Path(a.out).write_text(json.dumps(rep, indent=1))
        return
    from model_fixtures import EVERY_KIND
    dev = torch.device("cuda:0")
    rep = {"tolerance": f"|d| <= {ATOL} + {RTOL} |ref| (north_star)"}
    for name in (a.kinds or EVERY_KIND):
        rep[name] = measure(name, dev)
        print(name, json.dumps(rep[name]), flush=True)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
