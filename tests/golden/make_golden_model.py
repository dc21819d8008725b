"""End-to-end golden fixtures from the REFERENCE's forward() (dev container only).

    python tests/golden/make_golden_model.py [all | bench | geometry | real [name ...]]

Tiny-width LLaVA-OneVision teacher/student (real vocab 152064/151936, real 336x336 token
layout: 2 tiles, 1485 image tokens, L=1536) with seeded weights drawn by the build's own
ParamStore (CPU RNG, spec order) are loaded into transformers' model; the reference's
DT / LB / FB / BD module code (forward, compute_*_loss, contrastive_loss, hooks) runs the
step, autograd gives the student gradients.  Only outputs are committed
(tests/golden/model_*.npz).  Weights and inputs are regenerated from seeds in the tests.

`real`: the same with the REAL widths cut to 2 layers per tower (model_real_*.npz, bs 1):
SigLIP 1152/4304 with 16 heads of hd 72, Qwen2-7B 3584/18944 with 28q/4kv heads of hd 128,
Qwen2-0.5B 896/4864 with 14q/2kv heads of hd 64, the real vocabularies.
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(HERE))
import make_golden as MG  # noqa: E402
from oracle.model import hf5_key  # noqa: E402
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (  # noqa: E402
    ParamStore, real_width_config, tiny_config)
from model_fixtures import GRAD_SAMPLE, grad_sample_index  # noqa: E402

CONFIGS = {"tiny": (tiny_config(True), tiny_config(False)),
           "real2": (real_width_config(True, 2), real_width_config(False, 2))}
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import (  # noqa: E402
    synthetic_batch, synthetic_batch_mixed)

SEED_T, SEED_S, SEED_DATA = 1, 2, 0
B, L = 2, 1536


def tiny_state(teacher: bool, seed: int, cfg=None):
    P = ParamStore(cfg or tiny_config(teacher), "cpu")
    P.init_(seed, cpu_rng=True)
    return {k: v.float().clone() for k, v in P.state_dict().items()}


def hf_model(cfg, sd):
    from transformers import LlavaOnevisionConfig, LlavaOnevisionForConditionalGeneration
    V, T = cfg.vision, cfg.text
    hc = LlavaOnevisionConfig(
        vision_config=dict(model_type="siglip_vision_model", hidden_size=V.hidden, intermediate_size=V.inter,
                           num_hidden_layers=V.layers, num_attention_heads=V.heads, patch_size=V.patch,
                           image_size=V.image, vision_use_head=False, layer_norm_eps=V.eps),
        text_config=dict(model_type="qwen2", hidden_size=T.hidden, intermediate_size=T.inter,
                         num_hidden_layers=T.layers, num_attention_heads=T.heads, num_key_value_heads=T.kv_heads,
                         vocab_size=T.vocab, tie_word_embeddings=T.tie, rope_theta=T.rope_theta,
                         rms_norm_eps=T.eps, max_position_embeddings=4096),
        tie_word_embeddings=T.tie)
    m = LlavaOnevisionForConditionalGeneration(hc).float()
    sd5 = {hf5_key(k): v for k, v in sd.items()}
    missing, unexpected = m.load_state_dict(sd5, strict=False)
    assert not unexpected, unexpected
    assert all(k == "lm_head.weight" for k in missing), missing   # tied head
    return m


def batch_cpu(sizes=None, bs=B):
    """The 336x336 bench layout (B = 2, L = 1536), or with `sizes` a SUNRGBD-geometry batch
    (data.synthetic_batch_mixed: one image per sample at its own size, right padding)."""
    if sizes is None:
        b = synthetic_batch(bs, "cpu", L=L, seed=SEED_DATA, pixel_dtype=torch.bfloat16, cpu_rng=True)
    else:
        b = synthetic_batch_mixed(sizes, "cpu", seed=SEED_DATA, pixel_dtype=torch.bfloat16, cpu_rng=True)
    for k in ("rgb_pixel_values", "depth_pixel_values"):
        b[k] = b[k].float()
    return b


def hf5_to_445(name):
    for k445 in STUDENT_KEYS:
        if hf5_key(k445) == name:
            return k445
    return None


# rows of the student logits recorded in full (first / image / last text positions of each sample)
LOGIT_ROWS = (0, 23, 24, 700, 1508, 1509, 1534, 1535)
LOGIT_COL_STRIDE = 37      # ... at every 37th vocab column (4107 of 151936)


class _Recorder:
    """Captures the per-term values of the reference's forward without editing it: the
    HF models' outputs (forward hooks: logits, in-model CE), every F.kl_div the loss
    functions call (the KD term before its T^2 factor) and contrastive_loss's value."""

    def __init__(self):
        self.kl, self.ntx, self.out = [], [], {}

    def __enter__(self):
        import torch.nn.functional as F
        self._F = F
        self._kl = F.kl_div

        def kl_rec(*a, **k):
            v = self._kl(*a, **k)
            self.kl.append(float(v))
            return v
        F.kl_div = kl_rec
        return self

    def __exit__(self, *exc):
        self._F.kl_div = self._kl

    def hook(self, name):
        def fn(mod, args, out):
            self.out[name] = out
        return fn

    def wrap_contrastive(self, obj):
        orig = obj.contrastive_loss

        def rec(*a, **k):
            v = orig(*a, **k)
            self.ntx.append(float(v))
            return v
        obj.contrastive_loss = rec


def logit_stats(logits, rows=LOGIT_ROWS):
    """Per-row logsumexp and sum (fp64) of [B, L, V] logits, plus `rows` sampled at every
    LOGIT_COL_STRIDE-th column."""
    x = logits.detach().double()
    return (torch.logsumexp(x, -1).reshape(-1).numpy(), x.sum(-1).reshape(-1).numpy(),
            x[:, list(rows), ::LOGIT_COL_STRIDE].float().numpy())


_REF = {}


def _ref_classes():
    if not _REF:
        MG._install_stub()
        _REF.update(DT=MG._load("ref_dt", MG.DT_PATH), LB=MG._load("ref_lb", MG.LB_PATH),
                    FB=MG._load("ref_fb", MG.FB_PATH), BD=MG._load_bd())
    return _REF["DT"], _REF["LB"], _REF["FB"], _REF["BD"]


def run(kind, phase, teacher_sd, student_sd, out_name, sizes=None, model="tiny", bs=B):
    """model: "tiny" (tiny widths, 2 layers) or "real2" (the real widths, 2 layers per tower:
    modeling.real_width_config); the latter also records every parameter's gradient at
    GRAD_SAMPLE seeded positions (model_fixtures.grad_sample_index) for per-parameter cosines."""
    from transformers import LlavaOnevisionForConditionalGeneration  # noqa: F401
    DT, LB, FB, BD = _ref_classes()
    tcfg, scfg = CONFIGS[model]
    student = hf_model(scfg, student_sd)
    teacher = hf_model(tcfg, teacher_sd) if kind != "bd" else None
    batch = batch_cpu(sizes, bs)
    Bb, Lb = batch["depth_input_ids"].shape
    rows = LOGIT_ROWS if sizes is None else (0, 23, 24, Lb // 2, Lb - 28, Lb - 27, Lb - 2, Lb - 1)
    rec = _Recorder()
    student.register_forward_hook(rec.hook("student"))
    if teacher is not None:
        teacher.register_forward_hook(rec.hook("teacher"))
    T = 1.0
    with rec:
        if kind == "bd":
            obj = MG._bare(BD, model=student)
            student.train()
            loss = obj.training_step(batch, 0)
        else:
            cls, hp = {"dt": (DT, dict(T=0.8, gamma=0.8, soft_target_loss_weight=0.1, ce_loss_weight=0.5, phase=phase)),
                       "lb": (LB, dict(T=1, soft_target_loss_weight=0.5, ce_loss_weight=0.5)),
                       "fb": (FB, dict(T=0.8, soft_target_loss_weight=0.1, ce_loss_weight=0.8))}[kind]
            T = float(hp["T"])
            obj = MG._bare(cls, teacher_model=teacher, student_model=student, **hp)
            rec.wrap_contrastive(obj)
            teacher.eval()
            for p in teacher.parameters():
                p.requires_grad = False
            # the reference's own hook functions, at the transformers-5 module path (DT:110-121)
            teacher.model.vision_tower.post_layernorm.register_forward_hook(obj.hook_fn_teacher)
            student.model.vision_tower.post_layernorm.register_forward_hook(obj.hook_fn_student)
            if kind == "dt" and phase == 1:     # DT1T:105/111: freeze_student_language_layers
                for p in student.model.language_model.parameters():
                    p.requires_grad = False
                for p in student.lm_head.parameters():
                    p.requires_grad = False
            if kind == "dt" and phase == 2:     # DT2T:106/112: freeze_student_vision_layers
                for p in student.model.vision_tower.parameters():
                    p.requires_grad = False
            student.train()
            loss = obj.training_step(batch, 0)
    assert len(rec.kl) <= 1 and len(rec.ntx) <= 1, (rec.kl, rec.ntx)
    loss.backward()
    grads = {}
    for n, p in student.named_parameters():
        if p.grad is None:
            continue
        k445 = hf5_to_445(n) or ("language_model.model.embed_tokens.weight" if n == "lm_head.weight" else None)
        if k445 is None:
            continue
        g = p.grad.detach().double()
        if k445 in grads:
            raise RuntimeError(k445)
        grads[k445] = g
    so = rec.out["student"]
    out = dict(total=np.float64(loss.item()),
               # per-term values of the reference's own forward (NaN = the term is absent)
               kd_term=np.float64(rec.kl[0] * T * T if rec.kl else np.nan),     # kl_div(...) * T**2
               student_ce=np.float64(so.loss.item()),
               teacher_ce=np.float64(rec.out["teacher"].loss.item() if "teacher" in rec.out else np.nan),
               ntxent=np.float64(rec.ntx[0] if rec.ntx else np.nan))
    lse, rsum, srows = logit_stats(so.logits, rows)
    out.update(s_logit_lse=lse, s_logit_rowsum=rsum, s_logit_rows=srows, logit_rows=np.array(rows),
               logit_col_stride=np.int64(LOGIT_COL_STRIDE))
    if "teacher" in rec.out:
        tl, ts, _ = logit_stats(rec.out["teacher"].logits)
        out.update(t_logit_lse=tl, t_logit_rowsum=ts)
    names = sorted(grads)
    out["grad_names"] = np.array(names)
    out["grad_norms"] = np.array([float(grads[n].norm()) for n in names])
    out["grad_heads"] = np.stack([grads[n].reshape(-1)[:16].float().numpy() for n in names]) if names else np.zeros((0, 16))
    tot = sum(float(grads[n].pow(2).sum()) for n in names)
    out["grad_total_norm"] = np.float64(math_sqrt(tot))
    if model != "tiny":
        # [n_params, GRAD_SAMPLE], NaN past a small parameter's last element
        gs = np.full((len(names), GRAD_SAMPLE), np.nan, dtype=np.float32)
        for i, n in enumerate(names):
            v = grads[n].reshape(-1)[grad_sample_index(n, grads[n].numel())].float().numpy()
            gs[i, :v.size] = v
        out["grad_samples"] = gs
    meta = dict(kind=kind, phase=phase, B=Bb, L=Lb, seed_t=SEED_T, seed_s=SEED_S, seed_data=SEED_DATA, model=model)
    if sizes is not None:
        meta["sizes"] = [list(hw) for hw in sizes]
    np.savez_compressed(HERE / f"model_{out_name}.npz", meta=json.dumps(meta), **out)
    print(out_name, {k: float(out[k]) for k in ("total", "kd_term", "student_ce", "teacher_ce", "ntxent")},
          "grad norm", out["grad_total_norm"], "n_grads", len(names))


def math_sqrt(x):
    import math
    return math.sqrt(x)


STUDENT_KEYS = []


# real SUNRGBD geometry (SURVEY KAT 9, DM:127-146, DS:185-212): one 480x640 image (5 tiles,
# 2,929 image tokens, L = 2,980) — LoCa only works unpadded (KAT 2), so bs 1 — and a mixed,
# right-padded batch [336x336, 480x640] (pads labelled -100) for the kinds that accept pads
GEOMETRY = (
    ("lb", 0, "sun_lb", [(480, 640)]),
    ("dt", 1, "sun_dt1", [(480, 640)]),
    ("bd", 0, "mix_bd", [(336, 336), (480, 640)]),
    ("fb", 0, "mix_fb", [(336, 336), (480, 640)]),
    ("dt", 1, "mix_dt1", [(336, 336), (480, 640)]),
)


# the real widths at 2 layers per tower, bs 1, 336x336 (L = 1536): SigLIP hd 72, the teacher's
# hd 128 with GQA 28/4 at width 3584, the student's 14/2 at 896, the real MLP widths
REAL = (("lb", 0, "real_lb"), ("dt", 1, "real_dt1"), ("dt", 2, "real_dt2"), ("fb", 0, "real_fb"),
        ("dt", 3, "real_dt3"), ("bd", 0, "real_bd"))


def main_real(names):
    ssd = tiny_state(False, SEED_S, CONFIGS["real2"][1])
    tsd = tiny_state(True, SEED_T, CONFIGS["real2"][0])
    STUDENT_KEYS.extend(ssd.keys())
    for kind, phase, name in REAL:
        if names and name not in names:
            continue
        run(kind, phase, tsd, ssd, name, model="real2", bs=1)


def main():
    torch.set_num_threads(os.cpu_count())
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which == "real":
        return main_real(sys.argv[2:])
    ssd = tiny_state(False, SEED_S)
    tsd = tiny_state(True, SEED_T)
    STUDENT_KEYS.extend(ssd.keys())
    if which in ("all", "bench"):
        for kind, phase, name in (("lb", 0, "lb"), ("dt", 1, "dt1"), ("dt", 2, "dt2"), ("dt", 3, "dt3"),
                                  ("fb", 0, "fb"), ("bd", 0, "bd")):
            run(kind, phase, tsd, ssd, name)
    if which in ("all", "geometry"):
        for kind, phase, name, sizes in GEOMETRY:
            run(kind, phase, tsd, ssd, name, sizes)


if __name__ == "__main__":
    main()
