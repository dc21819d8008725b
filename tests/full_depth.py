"""Full-depth model parity of BASELINE config c1 (logit-based KD, LoCa T = 1; LB:29-33,
:125-169, :208-261): the HIP training_step of the drop-in module with the REAL 7B teacher and
0.5B student (all 26 + 28 / 26 + 24 layers, L = 1536, one 336x336 sample) against the pinned
CPU oracle (oracle/model.py, fp32 end to end as the reference's LB teacher and student) run on
the SAME weights (the device's bf16 flat buffers, copied to the host and widened to fp32) and
the same batch.  Shared by tests/test_full_depth_parity_gpu.py and tools/parity_report.py
--full-depth.  GPU only; ~40 GB of host memory for the oracle (weights + activations).

Measured (every value relative to the fp32 oracle, the tolerance of north_star |d| <= 1e-4 +
1e-3 |ref| where it applies):
  terms      KD term, student CE, teacher CE, total
  lse        per-row logsumexp of the student AND the teacher logits (all 1536 rows)
  logits     sampled rows of the student logits, split at the lm_head: the stored bf16 logits,
             the same GEMM with an fp32 output (no final rounding), and the floor a single bf16
             rounding of the reference's own lm_head input leaves
  grads      the gradient's total norm, per parameter group and per parameter (norm and
             cosine against the oracle's full fp32 gradient)
  floor      optionally the same oracle run in plain bf16 (weights and activations bf16), the
             yardstick where a figure misses the north-star
"""
from __future__ import annotations

import gc
import math
import time

import torch

S_NAME, T_NAME = "llava-hf/llava-onevision-qwen2-0.5b-ov-hf", "llava-hf/llava-onevision-qwen2-7b-ov-hf"
ATOL, RTOL = 1e-4, 1e-3
N_ROWS = 48            # sampled student-logit rows (all 151,936 columns each)


def _log(msg):
    print(f"[full_depth {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def _ns(got: float, ref: float) -> dict:
    d = abs(got - ref)
    return dict(got=got, ref=ref, abs=d, rel=d / abs(ref) if ref else None, ok=bool(d <= ATOL + RTOL * abs(ref)))


def _cmp_vec(got: torch.Tensor, ref: torch.Tensor) -> dict:
    """Elementwise: max |d|, max rel, fraction within the north-star."""
    got, ref = got.double().reshape(-1), ref.double().reshape(-1)
    d = (got - ref).abs()
    tol = ATOL + RTOL * ref.abs()
    return dict(max_abs=float(d.max()), max_rel=float((d / ref.abs().clamp_min(1e-30)).max()),
                frac_within=float((d <= tol).double().mean()), ok=bool((d <= tol).all()),
                rel_l2=float((got - ref).norm() / ref.norm()))


IMAGE_HW = [(336, 336)]   # the batch geometry of hip_step / oracle_step (sunrgbd(): 480x640)


def batch_cpu():
    """One sample: the 336x336 bench layout (L 1536, 2 tiles), or a real SUNRGBD image size
    (480x640: 5 tiles, 2,929 image tokens, L 2,980; SURVEY KAT 9, DS:185-212) when IMAGE_HW says so."""
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import (synthetic_batch,
                                                                                              synthetic_batch_mixed)
    if IMAGE_HW[0] == (336, 336):
        return synthetic_batch(1, "cpu", L=1536, seed=0, pixel_dtype=torch.bfloat16, cpu_rng=True)
    return synthetic_batch_mixed([IMAGE_HW[0]], "cpu", seed=0, pixel_dtype=torch.bfloat16, cpu_rng=True)


class geometry:
    """with geometry((480, 640)): hip_step / oracle_step on that image size."""

    def __init__(self, hw):
        self.hw, self.old = tuple(hw), None

    def __enter__(self):
        self.old, IMAGE_HW[0] = IMAGE_HW[0], self.hw
        return self

    def __exit__(self, *exc):
        IMAGE_HW[0] = self.old


def _to(b, dev):
    return {k: (v.to(dev) if torch.is_tensor(v) and k != "image_sizes" else v) for k, v in b.items()}


def group_of(name: str) -> str:
    """Parameter group: the per-layer tensors of one kind summed over layers."""
    for tag in ("embed_tokens", "lm_head", "model.norm.weight", "patch_embedding", "position_embedding",
                "post_layernorm", "multi_modal_projector", "image_newline"):
        if tag in name:
            return name
    return ".".join(p for p in name.split(".") if not p.isdigit())


def row_index(L: int | None = None, n: int = N_ROWS):
    if L is None:
        L = 1536 if IMAGE_HW[0] == (336, 336) else int(batch_cpu()["rgb_input_ids"].shape[1])
    g = torch.Generator().manual_seed(1234)
    return torch.randperm(L, generator=g)[:n].sort().values


def hip_step(dev, teacher_residual_f32: bool = False, keep_weights: bool = True, teacher_fp8: bool | str = False):
    """One training_step + backward of LogitBasedKD at full size, bs 1.  Returns (results on
    the host, teacher state_dict, student state_dict) -- the weights as fp32 host tensors.
    teacher_fp8: the e4m3 teacher of BASELINE config c4 (a modeling.FP8_FAMILIES policy), on the
    same (seeded) bf16 weights, quantised after the load."""
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops
    m = K.LogitBasedKD(S_NAME, T_NAME, teacher_residual_f32=teacher_residual_f32, teacher_fp8=teacher_fp8)
    bc = batch_cpu()
    b = _to(bc, dev)
    m.keep_logits = True
    loss = m.training_step(b, 0)
    loss.backward()
    m.check_errors()
    torch.cuda.synchronize()
    s3, t3 = m.last_logits
    kd, ce, tce, tot = m.last_terms.tolist()
    rows = row_index()
    res = dict(terms=dict(kd_term=kd, student_ce=ce, teacher_ce=tce, total=float(loss.item())),
               weights_checksum=[float(m.teacher_model.P.flat[:1 << 22].float().sum()),
                                 float(m.student_model.P.flat[:1 << 22].float().sum())],
               s_lse=torch.logsumexp(s3[0].double(), -1).cpu(),
               t_lse=torch.logsumexp(t3[0].double(), -1).cpu(),
               s_rows=s3[0, rows.to(dev)].float().cpu(),
               t_rows=t3[0, rows.to(dev), :s3.shape[-1]].float().cpu())
    m.last_logits = None
    del s3, t3
    # the lm_head again on the same final-norm hidden state with an fp32 output: the logits before
    # their bf16 rounding (the forward is deterministic and no optimizer step ran)
    s = m.student_model
    fwd = s.forward(b["depth_input_ids"], b["depth_pixel_values"], b["image_sizes"])
    hn = fwd["hn"][rows.to(dev)].contiguous()
    res["s_rows_f32"] = ops.gemm(hn, s.lm_head_weight(), out_dtype=torch.float32).cpu()
    res["hn_rows"] = hn.float().cpu()
    del fwd, hn
    P = s.P
    g = P.grad
    torch.cuda.synchronize()
    grads = {}
    for spec in P.specs:
        v = P.view(spec.name, g)
        if spec.ckpt_shape is not None:
            v = v[:, :math.prod(spec.ckpt_shape[1:])].reshape(spec.ckpt_shape)
        grads[spec.name] = v.cpu().clone()
    res["grads"] = grads
    tsd = ssd = None
    if keep_weights:
        tsd = {k: v.detach().float().cpu() for k, v in m.teacher_model.P.state_dict().items()}
        ssd = {k: v.detach().float().cpu() for k, v in P.state_dict().items()
               if k != "language_model.lm_head.weight"}     # tied: one tensor, as transformers
    del m, loss, b
    gc.collect()
    torch.cuda.empty_cache()
    return res, tsd, ssd


def oracle_step(tsd, ssd, dtype=torch.float32):
    """The pinned CPU oracle's LB step (compute_loca_loss at T = 1 + the student CE, LB:164-165)
    on the same weights, in `dtype`; the student gradient by autograd."""
    from oracle import kd_losses as KL
    from oracle.model import OracleLlava
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import STUDENT_05B, TEACHER_7B
    b = batch_cpu()
    for k in ("rgb_pixel_values", "depth_pixel_values"):
        b[k] = b[k].to(dtype)
    tw = {k: v.to(dtype) for k, v in tsd.items()}
    sw = {k: v.detach().to(dtype).requires_grad_(True) for k, v in ssd.items()}   # leaves (fp32: no copy)
    teacher, student = OracleLlava(tw, TEACHER_7B), OracleLlava(sw, STUDENT_05B)
    with torch.no_grad():
        t_logits, _ = teacher(b["rgb_input_ids"], b["rgb_pixel_values"], b["image_sizes"])
    del teacher, tw
    gc.collect()
    s_logits, _ = student(b["depth_input_ids"], b["depth_pixel_values"], b["image_sizes"])
    hn = student.last_hn.detach()
    labels = b["labels"]
    kd = KL.loca_kd_term(t_logits, s_logits, labels, T=KL.LB_HPARAMS["T"], alpha=KL.LB_HPARAMS["alpha"])
    ce = KL.causal_lm_ce(s_logits, labels)
    tce = KL.causal_lm_ce(t_logits, labels)
    total = kd + ce
    total.float().backward()
    rows = row_index()
    res = dict(terms=dict(kd_term=float(kd.detach()), student_ce=float(ce.detach()), teacher_ce=float(tce),
                          total=float(total.detach())),
               s_lse=torch.logsumexp(s_logits[0].detach().double(), -1),
               t_lse=torch.logsumexp(t_logits[0].double(), -1),
               s_rows=s_logits[0, rows].detach().float(),
               t_rows=t_logits[0, rows, :s_logits.shape[-1]].float(),
               hn_rows=hn[0, rows].float(),
               grads={k: v.grad for k, v in sw.items() if v.grad is not None})
    del s_logits, t_logits, kd, ce, tce, total, student
    gc.collect()
    return res


KINDS = {"lb": ("lb", 0), "dt1": ("dt", 1), "dt2": ("dt", 2), "dt3": ("dt", 3), "fb": ("fb", 0), "bd": ("bd", 0)}


def _module(kind: str, phase: int, teacher_fp8: bool | str = False):
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
    if kind == "lb":
        return K.LogitBasedKD(S_NAME, T_NAME, teacher_fp8=teacher_fp8)
    if kind == "fb":
        return K.FeatureBasedKD(S_NAME, T_NAME, teacher_fp8=teacher_fp8)
    if kind == "bd":
        return K.LlavaOnevisionModule(S_NAME)
    m = K.OnlineKnowledgeDistillationLLavaOneVision(S_NAME, T_NAME, phase=phase, teacher_fp8=teacher_fp8)
    if phase == 1:
        m.freeze_student_language_layers()       # DT1T:105/111
    if phase == 2:
        m.freeze_student_vision_layers()         # DT2T:106/112
    return m


def hip_step_kind(dev, name: str, teacher_fp8: bool | str = False, detail: bool = False):
    """One training_step + backward of module `name` (KINDS: the reference's DT phases 1-3, LB, FB,
    BD) at full size, bs 1: the total, the student logits' per-row logsumexp, the trainable
    parameters' gradients, and both models' weights (fp32 host tensors) for the oracle.
    teacher_fp8: the e4m3 teacher (a modeling.FP8_FAMILIES policy; BASELINE config c4) on the same
    seeded bf16 weights.  detail: also the fused kernel's KD term, student CE and teacher CE, and
    the teacher logits' per-row logsumexp."""
    kind, phase = KINDS[name]
    m = _module(kind, phase, teacher_fp8)
    b = _to(batch_cpu(), dev)
    m.keep_logits = True
    loss = m.training_step(b, 0)
    loss.backward()
    m.check_errors()
    torch.cuda.synchronize()
    s3, t3 = m.last_logits
    res = dict(terms=dict(total=float(loss.item())), s_lse=torch.logsumexp(s3[0].double(), -1).cpu())
    if detail and t3 is not None:
        kd, ce, tce, _ = m.last_terms.tolist()
        res["terms"].update(kd_term=kd, student_ce=ce, teacher_ce=tce)
        res["t_lse"] = torch.logsumexp(t3[0].double(), -1).cpu()
    m.last_logits = None
    del s3, t3
    P = m.student_model.P
    g = P.grad
    grads = {}
    for spec in P.specs:
        v = P.view(spec.name, g)
        if spec.ckpt_shape is not None:
            v = v[:, :math.prod(spec.ckpt_shape[1:])].reshape(spec.ckpt_shape)
        grads[spec.name] = v.cpu().clone()
    res["grads"] = grads
    tsd = None if m.teacher_model is None else {k: v.detach().float().cpu() for k, v in m.teacher_model.P.state_dict().items()}
    ssd = {k: v.detach().float().cpu() for k, v in P.state_dict().items() if k != "language_model.lm_head.weight"}
    del m, loss, b
    gc.collect()
    torch.cuda.empty_cache()
    return res, tsd, ssd


def oracle_step_kind(tsd, ssd, name: str, detail: bool = False):
    """The pinned fp32 oracle's forward(batch) total of module `name` (oracle.model.kd_step_losses: DT:250-260,
    LB:164-165, FB:161-165, BD:90-101) on the same weights; the gradient of the trainable parameters (the
    reference's freezes, tests/golden/model_fixtures.frozen) by autograd.  detail: also the KD term of the
    module's variant (LoCa DT:141-194 / KL DT:330-343 / log-target KL FB:205-219), the student and the
    teacher CE, and the teacher logits' per-row logsumexp."""
    from oracle.model import OracleLlava, kd_step_losses
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import STUDENT_05B, TEACHER_7B
    kind, phase = KINDS[name]
    tv, tp, tl = (True, True, False) if (kind, phase) == ("dt", 1) else \
        ((False, True, True) if (kind, phase) == ("dt", 2) else (True, True, True))
    b = batch_cpu()
    for k in ("rgb_pixel_values", "depth_pixel_values"):
        b[k] = b[k].float()
    sw = {}
    for k, v in ssd.items():
        train = tl if k.startswith("language_model") else \
            (tp if (k.startswith("multi_modal") or k == "image_newline") else tv)
        sw[k] = v.detach().float().requires_grad_(train)
    student = OracleLlava(sw, STUDENT_05B)
    teacher = None if tsd is None else OracleLlava({k: v.float() for k, v in tsd.items()}, TEACHER_7B)
    total, aux = kd_step_losses(kind, teacher, student, b, phase=phase)
    total.float().backward()
    res = dict(terms=dict(total=float(total.detach())),
               s_lse=torch.logsumexp(aux["s_logits"][0].detach().double(), -1),
               grads={k: v.grad for k, v in sw.items() if v.grad is not None})
    if detail and teacher is not None:
        from oracle import kd_losses as KL
        s_l, t_l, labels = aux["s_logits"].detach(), aux["t_logits"], b["labels"]
        h = KL.DT_HPARAMS if kind == "dt" else (KL.LB_HPARAMS if kind == "lb" else KL.FB_HPARAMS)
        if kind == "fb":
            kd = KL.kl_logtarget_term(t_l, s_l, h["T"])
        elif (kind, phase) == ("dt", 1):
            kd = KL.kl_mean_term(t_l, s_l, h["T"])
        else:
            kd = KL.loca_kd_term(t_l, s_l, labels, T=h["T"], alpha=h["alpha"])
        res["terms"].update(kd_term=float(kd), student_ce=float(KL.causal_lm_ce(s_l, labels)),
                            teacher_ce=float(KL.causal_lm_ce(t_l, labels)))
        res["t_lse"] = torch.logsumexp(t_l[0].double(), -1)
        del s_l, t_l, kd
    del total, aux, student, teacher
    gc.collect()
    return res


def measure_kinds(dev, names) -> dict:
    """Full-depth parity of each module in `names` against the fp32 oracle on its own weights."""
    rep = {"tolerance": f"|d| <= {ATOL} + {RTOL} |ref| (north_star); gradient total norm rel <= {RTOL}",
           "batch": "bs 1, L 1536, one 336x336 image (2 tiles); full depth: SigLIP 26 + Qwen2 28 / 24 layers"}
    for name in names:
        t0 = time.time()
        _log(f"{name}: HIP step")
        hip, tsd, ssd = hip_step_kind(dev, name)
        _log(f"{name}: fp32 oracle step ({torch.get_num_threads()} threads)")
        ref = oracle_step_kind(tsd, ssd, name)
        rep[name] = compare(hip, ref, None)
        rep[name]["seconds"] = round(time.time() - t0, 1)
        del hip, ref, tsd, ssd
        gc.collect()
    return rep


def _rel_l2(a, b) -> float:
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a - b).norm() / b.norm())


def measure_depth_profile(dev, vision_depths=(1, 4, 8, 13, 17, 21, 26), text_depths=(1, 4, 8, 12, 16, 20, 24)) -> dict:
    """Where along the student's towers the final hidden state's error against the fp32 oracle is
    added (DT:232-240): the 0.5B student of c1 (seeded weights, one 336x336
    sample) cut to `dv` SigLIP and `dt` Qwen2 layers -- the same weights, so the cut model's
    outputs ARE the full model's hidden states at that depth, passed through the final norm --
    on the HIP path (bf16 GEMMs, fp32 residual streams) and through the fp32 oracle.
      vision[dv]: rel-L2 of the post-LN hook output (post_layernorm of SigLIP layer dv's output)
      text[dt]:   rel-L2 of hn = norm(Qwen2 layer dt's output), with the full 26-layer SigLIP
    and, as the yardstick, one bf16 rounding of the oracle's own tensor (the floor of any bf16
    output).  The projector sits between them (text[1] - vision[26])."""
    from dataclasses import replace
    from oracle.model import OracleLlava
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (
        STUDENT_05B, LlavaOnevisionModel)
    full = LlavaOnevisionModel(STUDENT_05B, dev, trainable=True, seed=2)
    sd = {k: v.detach().float().cpu() for k, v in full.P.state_dict().items() if k != "language_model.lm_head.weight"}
    del full
    gc.collect()
    torch.cuda.empty_cache()
    bc = batch_cpu()
    b = _to(bc, dev)
    bo = dict(bc)
    for k in ("rgb_pixel_values", "depth_pixel_values"):
        bo[k] = bo[k].float()

    def keep(cfg):
        Vl, Tl = cfg.vision.layers, cfg.text.layers
        out = {}
        for k, v in sd.items():
            if ".encoder.layers." in k and int(k.split(".encoder.layers.")[1].split(".")[0]) >= Vl:
                continue
            if "language_model.model.layers." in k and int(k.split("language_model.model.layers.")[1].split(".")[0]) >= Tl:
                continue
            out[k] = v
        return out

    def one(dv, dt):
        cfg = replace(STUDENT_05B, vision=replace(STUDENT_05B.vision, layers=dv),
                      text=replace(STUDENT_05B.text, layers=dt))
        w = keep(cfg)
        m = LlavaOnevisionModel(cfg, dev, trainable=True)
        m.P.load_state_dict({k: v.to(dev) for k, v in w.items()}, strict=False)
        f = m.forward(b["depth_input_ids"], b["depth_pixel_values"], b["image_sizes"], want_post_ln=True)
        torch.cuda.synchronize()
        hn, post = f["hn"].float().cpu(), f["post_ln"].float().cpu()
        del f, m
        torch.cuda.empty_cache()
        o = OracleLlava(w, cfg)
        with torch.no_grad():
            _, opost = o(bo["depth_input_ids"], bo["depth_pixel_values"], bo["image_sizes"])
        ohn = o.last_hn[0]
        opost = opost.reshape(post.shape)
        return dict(hn=_rel_l2(hn, ohn), hn_floor=_rel_l2(ohn.bfloat16(), ohn),
                    post_ln=_rel_l2(post, opost), post_ln_floor=_rel_l2(opost.bfloat16(), opost))

    rep = {"config": "c1 student (0.5B: SigLIP 26 + Qwen2 24), seeded weights, bs 1, L 1536, 336x336; HIP vs the fp32 "
                     "oracle on the same weights, the models cut to the listed depths",
           "vision": {}, "text": {}}
    for dv in vision_depths:
        _log(f"depth profile: SigLIP {dv}")
        r = one(dv, 1)
        rep["vision"][str(dv)] = dict(post_ln_rel_l2=r["post_ln"], floor=r["post_ln_floor"])
    for dt in text_depths:
        _log(f"depth profile: Qwen2 {dt}")
        r = one(STUDENT_05B.vision.layers, dt)
        rep["text"][str(dt)] = dict(hn_rel_l2=r["hn"], floor=r["hn_floor"])
    return rep


C4_FP8_TOL = 1e-2   # the fp8 (e4m3) teacher's stated tolerance on the teacher-side terms


def measure_c4(dev, policy: str = "lm_mlp") -> dict:
    """BASELINE config c4's own module at full depth: double-trouble phase 3 (DT:257-260: 0.8 (LoCa
    at T = 0.8 + CE) + 0.2 CE) with the fp8 (e4m3) teacher `policy`, bs 1, against the fp32 oracle
    on the same (bf16-valued) weights -- the fp8 teacher's distance from the reference's fp32
    teacher, measured on the configuration c4 runs."""
    t0 = time.time()
    _log(f"c4: HIP step (DT phase 3, fp8 teacher {policy})")
    hip, tsd, ssd = hip_step_kind(dev, "dt3", teacher_fp8=policy, detail=True)
    _log(f"c4: fp32 oracle step ({torch.get_num_threads()} threads)")
    ref = oracle_step_kind(tsd, ssd, "dt3", detail=True)
    del tsd, ssd
    gc.collect()
    r = compare(hip, ref, None)
    r["config"] = (f"c4: DT phase 3 (LoCa T = 0.8), fp8 e4m3 teacher ({policy}), bs 1, L 1536, 336x336, full depth "
                   "(SigLIP 26 + Qwen2 28 / 24 layers)")
    r["tolerance"] = (f"north_star |d| <= {ATOL} + {RTOL} |ref| on the student CE, the total, every student lse row and "
                      f"the gradient total norm; rel <= {C4_FP8_TOL} on the KD term and the teacher CE (the fp8 teacher)")
    r["seconds"] = round(time.time() - t0, 1)
    return r


def compare(hip: dict, ref: dict, W: torch.Tensor | None = None) -> dict:
    """Every figure of `hip` against `ref` (both from hip_step / oracle_step)."""
    out = {"terms": {k: _ns(hip["terms"][k], ref["terms"][k]) for k in ref["terms"]}}
    if "weights_checksum" in hip:
        out["weights_checksum"] = hip["weights_checksum"]
    out["s_lse"] = _cmp_vec(hip["s_lse"], ref["s_lse"])
    if "t_lse" in hip and "t_lse" in ref:
        out["t_lse"] = _cmp_vec(hip["t_lse"], ref["t_lse"])
    if "s_rows" in hip and "s_rows" in ref:
        out["s_logits_rows"] = _cmp_vec(hip["s_rows"], ref["s_rows"])
        out["t_logits_rows"] = _cmp_vec(hip["t_rows"], ref["t_rows"])
    if "s_rows_f32" in hip:
        out["s_logits_rows_f32_out"] = _cmp_vec(hip["s_rows_f32"], ref["s_rows"])
    if "hn_rows" in hip and "hn_rows" in ref:
        out["hn_rows_rel_l2"] = float((hip["hn_rows"].double() - ref["hn_rows"].double()).norm()
                                      / ref["hn_rows"].double().norm())
    if W is not None and "hn_rows" in ref:
        # one bf16 rounding of the REFERENCE's own lm_head input, fp64 product: the floor of any
        # bf16-input lm_head, whatever happened upstream
        one = ref["hn_rows"].bfloat16().double() @ W.double().t()
        out["s_logits_rows_floor_bf16_input"] = _cmp_vec(one, ref["s_rows"])
    # gradients: total norm, per group, per parameter
    hg, rg = hip["grads"], ref["grads"]
    names = [n for n in rg]
    tot_h = math.sqrt(sum(float(hg[n].double().pow(2).sum()) for n in names))
    tot_r = math.sqrt(sum(float(rg[n].double().pow(2).sum()) for n in names))
    out["grad_total_norm"] = dict(got=tot_h, ref=tot_r, rel=(tot_h - tot_r) / tot_r,
                                  ok=bool(abs(tot_h - tot_r) <= RTOL * tot_r))
    groups = {}
    per = {}
    for n in names:
        a, r = hg[n].double().reshape(-1), rg[n].double().reshape(-1)
        an, rn = float(a.norm()), float(r.norm())
        cos = float((a @ r) / (an * rn + 1e-300))
        err = float((a - r).norm())
        per[n] = dict(ref_norm=rn, norm_rel=(an / rn - 1) if rn > 0 else an, cos=cos, err_rel=err / rn if rn else err)
        gr = groups.setdefault(group_of(n), [0.0, 0.0, 0.0])
        gr[0] += rn * rn
        gr[1] += an * an
        gr[2] += err * err
    out["grad_groups"] = {k: dict(ref_norm=math.sqrt(v[0]), norm_rel=math.sqrt(v[1] / v[0]) - 1 if v[0] else None,
                                  err_rel=math.sqrt(v[2] / v[0]) if v[0] else None)
                          for k, v in sorted(groups.items())}
    out["grad_params"] = per
    worst = sorted(per.items(), key=lambda kv: -abs(kv[1]["err_rel"]))[:8]
    out["grad_params_worst"] = {k: v for k, v in worst}
    out["grad_params_min_cos"] = min(v["cos"] for v in per.values() if v["ref_norm"] > 0)
    return out


def measure(dev, floor: bool = False, teacher_stream_ab: bool = False, teacher_fp8: str | None = None) -> dict:
    """The whole report: HIP (default teacher stream) vs the fp32 oracle; optionally the plain
    bf16 oracle (floor), the HIP step with the teacher's Qwen2 residual stream in fp32, and the
    HIP step with the fp8 (e4m3) teacher of config c4 (policy `teacher_fp8`) against the same fp32
    reference -- the fp8 teacher's full-depth distance from the reference, not from the bf16 teacher."""
    t0 = time.time()
    _log("HIP step (teacher Qwen2 stream bf16, the default)")
    hip, tsd, ssd = hip_step(dev, teacher_residual_f32=False)
    W = ssd["language_model.model.embed_tokens.weight"]
    hip32 = None
    if teacher_stream_ab:
        _log("HIP step (teacher Qwen2 stream fp32)")
        hip32, _, _ = hip_step(dev, teacher_residual_f32=True, keep_weights=False)
    hip8 = None
    if teacher_fp8:
        _log(f"HIP step (fp8 e4m3 teacher, policy {teacher_fp8})")
        hip8, _, _ = hip_step(dev, keep_weights=False, teacher_fp8=teacher_fp8)
    _log(f"fp32 oracle step on the same weights ({torch.get_num_threads()} threads)")
    ref = oracle_step(tsd, ssd, torch.float32)
    rep = {"config": "c1: LogitBasedKD (LoCa T = 1), bs 1, L 1536, 336x336, full depth (SigLIP 26 + Qwen2 28 / 24 layers)",
           "tolerance": f"|d| <= {ATOL} + {RTOL} |ref| (north_star); gradient total norm rel <= {RTOL}",
           "reference": "oracle/model.py + oracle/kd_losses.py in fp32 on the device's bf16 weights widened to fp32",
           "hip": compare(hip, ref, W)}
    if hip32 is not None:
        rep["hip_teacher_stream_f32"] = compare(hip32, ref, W)
        del hip32
    if hip8 is not None:
        rep["hip_teacher_fp8"] = compare(hip8, ref, W)
        rep["hip_teacher_fp8"]["policy"] = teacher_fp8
        del hip8
    if floor:
        _log("bf16 oracle step (the floor)")
        fl = oracle_step(tsd, ssd, torch.bfloat16)
        fl["grads"] = {k: v.float() for k, v in fl["grads"].items()}
        rep["bf16_floor"] = compare(fl, ref, None)
        del fl
    rep["seconds"] = round(time.time() - t0, 1)
    _log(f"done in {rep['seconds']} s")
    return rep
