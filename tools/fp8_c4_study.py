"""Why the c4 fp8 teacher's KD term moves: LoCa top-2 flips vs smooth probability change.

    python tools/fp8_c4_study.py [--seeds 0 1 2 3] [--batch 8] [--out gpurun_out/fp8_c4.json]
    KDSTEP_LIB=tools/ab/libkdstep_ab.so KD_GEMM_STAGGER=0 python tools/fp8_c4_study.py ...   (stagger off)

BASELINE config c4 = double-trouble phase 3 (DT:257-260: 0.8 (LoCa + CE) + 0.2 CE, LoCa at
T = 0.8, DT:141-194) with the e4m3 teacher MLPs.  For each seeded c4 batch (bs 8, the fresh
random-init models, no optimizer step) the module's forward runs with three teachers on the
same weights: fp8 (lm_mlp), bf16 (default), and bf16 with the fp32 Qwen2 residual stream (a
control: a perturbation of the bf16 teacher by accumulation / rounding order only).

Per pair (x, bf16) it reports the fused kernel's KD term and teacher CE, and from the teacher
logits: the rows whose LoCa second index k = topk(p_T, 2)[1] (DT:170-171) differs, the
symmetric difference of the klogit column sets, and |labels ∩ klogits| -- the label columns
whose global override X is replaced by a klogit override Y (KAT 1: klogits are written second).
The KD term is then split on the GPU (oracle arithmetic, test-infrastructure use) into
  flips   = KD(bf16 probs, x's k) - KD(bf16 probs, bf16's k)
  smooth  = KD(x probs, x's k) - KD(bf16 probs, x's k)
so the move of the term is attributed to the discrete override-set change or to the teacher's
probabilities themselves.  GPU only.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def _log(msg):
    print(f"[fp8_c4 {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def second_index(t, V):
    """DT:170-171 on the teacher logits (softmax at T keeps the order): lowest index on ties."""
    import torch
    v = t[..., :V]
    i1 = torch.argmax(v, dim=-1, keepdim=True)
    return torch.argmax(v.scatter(-1, i1, float("-inf")), dim=-1)


def loca_kd(t, s, labels, k, T):
    from oracle.kd_losses import loca_kd_term_rows
    return loca_kd_term_rows(t, s, labels, T, k=k)


def run(args):
    import torch
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    dev = torch.device("cuda", 0)
    S, T_ = "llava-hf/llava-onevision-qwen2-0.5b-ov-hf", "llava-hf/llava-onevision-qwen2-7b-ov-hf"
    m = K.OnlineKnowledgeDistillationLLavaOneVision(S, T_, phase=3, teacher_fp8="lm_mlp")
    variant, T = m._loss_spec()[:2]
    m.keep_logits = True
    rep = dict(config="c4: DT phase 3 (LoCa T = 0.8), bs %d, fresh random-init models, no optimizer step" % args.batch,
               stagger_env=__import__("os").environ.get("KD_GEMM_STAGGER"),
               lib=__import__("os").environ.get("KDSTEP_LIB", "product libkdstep.so"), seeds={})
    for seed in args.seeds:
        b = synthetic_batch(args.batch, dev, L=1536, seed=seed)
        V = None
        arms = {}
        for arm in ("fp8", "bf16", "bf16_f32stream"):
            if arm == "fp8":
                m.teacher_model.enable_fp8("lm_mlp")
                m.teacher_model.set_lm_stream_f32(False)
            elif arm == "bf16":
                m.teacher_model.disable_fp8()
            else:
                m.teacher_model.set_lm_stream_f32(True)
            with torch.no_grad():
                m.forward(b)
            torch.cuda.synchronize()
            s3, t3 = m.last_logits
            m.last_logits = None
            V = s3.shape[-1]
            arms[arm] = dict(terms=m.last_terms.tolist(), t=t3.clone(), k=second_index(t3, V))
            if arm == "bf16":
                s_ref = s3.clone()
            del s3, t3
        m.teacher_model.set_lm_stream_f32(False)
        m.teacher_model.enable_fp8("lm_mlp")
        labels = b["labels"]
        lab_set = torch.unique(labels.reshape(-1))
        base = arms["bf16"]
        kd_b = loca_kd(base["t"], s_ref, labels, base["k"], T)
        out = dict(label_columns=int(lab_set.numel()), kd_oracle_bf16=kd_b, kernel_terms_bf16=base["terms"])
        for arm in ("fp8", "bf16_f32stream"):
            a = arms[arm]
            kset_a, kset_b = torch.unique(a["k"]), torch.unique(base["k"])
            sym = int(torch.cat([kset_a, kset_b]).unique().numel() * 2 - kset_a.numel() - kset_b.numel())
            coll_a = int(torch.isin(kset_a, lab_set).sum())
            coll_b = int(torch.isin(kset_b, lab_set).sum())
            kd_a = loca_kd(a["t"], s_ref, labels, a["k"], T)
            kd_flip = loca_kd(base["t"], s_ref, labels, a["k"], T)   # bf16 probs, this arm's top-2
            rel = lambda x, y: (x - y) / y if y else None
            out[arm] = dict(
                kernel_terms=a["terms"],
                kernel_kd_rel_vs_bf16=rel(a["terms"][0], base["terms"][0]),
                kernel_teacher_ce_rel_vs_bf16=rel(a["terms"][2], base["terms"][2]),
                teacher_logits_rel_l2=float((a["t"].float() - base["t"].float()).norm() / base["t"].float().norm()),
                second_index_rows_flipped=int((a["k"] != base["k"]).sum()), rows=int(a["k"].numel()),
                klogit_columns=int(kset_a.numel()), klogit_columns_bf16=int(kset_b.numel()),
                klogit_columns_symdiff=sym, label_cols_overridden_by_klogits=coll_a,
                label_cols_overridden_by_klogits_bf16=coll_b,
                kd_oracle=kd_a, kd_oracle_rel_vs_bf16=rel(kd_a, kd_b),
                kd_split=dict(flips=rel(kd_flip, kd_b), smooth=rel(kd_a, kd_flip)))
            _log(f"seed {seed} {arm}: KD rel {out[arm]['kernel_kd_rel_vs_bf16']:+.5f} (oracle {out[arm]['kd_oracle_rel_vs_bf16']:+.5f}; "
                 f"flips {out[arm]['kd_split']['flips']:+.5f} smooth {out[arm]['kd_split']['smooth']:+.5f}), "
                 f"rows flipped {out[arm]['second_index_rows_flipped']}, label cols overridden {coll_a} vs {coll_b}")
        rep["seeds"][str(seed)] = out
        del arms, base, s_ref
        torch.cuda.empty_cache()
    for arm in ("fp8", "bf16_f32stream"):
        v = [abs(rep["seeds"][s][arm]["kernel_kd_rel_vs_bf16"]) for s in rep["seeds"]]
        rep[f"{arm}_kd_rel_abs"] = dict(values=v, max=max(v), mean=sum(v) / len(v))
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3])
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rep = run(a)
    s = json.dumps(rep, indent=1)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(s)
    print(s)


if __name__ == "__main__":
    main()
