"""Shared helpers for the end-to-end fixtures (tests/golden/model_*.npz): tiny widths, and the
real widths at 2 layers per tower (model_real_*.npz)."""
from __future__ import annotations

import json
import math
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
KINDS = {"lb": ("lb", 0), "dt1": ("dt", 1), "dt2": ("dt", 2), "dt3": ("dt", 3), "fb": ("fb", 0), "bd": ("bd", 0)}
# real SUNRGBD geometry (make_golden_model.GEOMETRY): 480x640 at bs 1, mixed [336^2, 480x640] right-padded
GEOMETRY_KINDS = {"sun_lb": ("lb", 0), "sun_dt1": ("dt", 1), "mix_bd": ("bd", 0), "mix_fb": ("fb", 0),
                  "mix_dt1": ("dt", 1)}
ALL_KINDS = {**KINDS, **GEOMETRY_KINDS}
# the real widths at 2 layers per tower (make_golden_model.REAL; bs 1, 336x336)
REAL_KINDS = {"real_lb": ("lb", 0), "real_dt1": ("dt", 1), "real_dt2": ("dt", 2), "real_fb": ("fb", 0),
              "real_dt3": ("dt", 3), "real_bd": ("bd", 0)}
EVERY_KIND = {**ALL_KINDS, **REAL_KINDS}
GRAD_SAMPLE = 4096   # gradient entries recorded per parameter in the real-width fixtures


def grad_sample_index(name: str, numel: int, k: int = GRAD_SAMPLE):
    """The positions (into the flattened reference-shape gradient) at which a real-width
    fixture records parameter `name`'s gradient: all of them for small parameters, else k
    draws from a generator seeded by the name (sorted; repeats allowed)."""
    import zlib
    if numel <= k:
        return torch.arange(numel)
    g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
    return torch.randint(0, numel, (k,), generator=g).sort().values


def model_config(meta, teacher: bool):
    """The architecture a fixture was generated with (meta["model"]: tiny | real2)."""
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (real_width_config,
                                                                                                    tiny_config)
    if meta.get("model", "tiny") == "real2":
        return real_width_config(teacher, 2)
    return tiny_config(teacher)


def module_names(meta):
    """(student, teacher) model names of the drop-in module for a fixture (kd_module.MODEL_CONFIGS)."""
    return ("real2-student", "real2-teacher") if meta.get("model", "tiny") == "real2" else ("tiny-student",
                                                                                             "tiny-teacher")


def load(name):
    z = np.load(HERE / f"model_{name}.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return meta, {k: z[k] for k in z.files if k != "meta"}


def tiny_weights(teacher: bool, seed: int, cfg=None):
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import ParamStore, tiny_config
    P = ParamStore(cfg or tiny_config(teacher), "cpu")
    P.init_(seed, cpu_rng=True)
    sd = {k: v.float().clone() for k, v in P.state_dict().items()}
    if P.cfg.text.tie:   # one tensor for embed_tokens and the tied lm_head (as in transformers)
        del sd["language_model.lm_head.weight"]
    return sd


def batch(meta, device="cpu"):
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import (synthetic_batch,
                                                                                                synthetic_batch_mixed)
    if "sizes" in meta:
        return synthetic_batch_mixed([tuple(hw) for hw in meta["sizes"]], device, seed=meta["seed_data"],
                                     pixel_dtype=torch.bfloat16, cpu_rng=True)
    return synthetic_batch(meta["B"], device, L=meta["L"], seed=meta["seed_data"], pixel_dtype=torch.bfloat16,
                           cpu_rng=True)


def frozen(kind, phase):
    """(vision, projector, language) trainable flags as the reference's train scripts set them."""
    if kind == "dt" and phase == 1:
        return True, True, False      # DT1T:105/111 freeze_student_language_layers
    if kind == "dt" and phase == 2:
        return False, True, True      # DT2T:106/112 freeze_student_vision_layers
    return True, True, True


def oracle_grads(name, dtype=torch.float32, with_logits=False):
    """Run the CPU oracle step for fixture `name`; returns (total, {param: grad}).
    dtype=torch.bfloat16: the same restatement with bf16 weights and activations (torch
    autograd on the CPU) — how far a plain bf16 run of the reference's arithmetic lands
    from its fp32 values, the yardstick for the HIP path's bf16 deltas."""
    from oracle.model import OracleLlava, kd_step_losses
    meta, _ = load(name)
    # with_logits: also return the student logits (detached, [B, L, V]) as a third value
    kind, phase = EVERY_KIND[name]
    scfg, tcfg = model_config(meta, False), model_config(meta, True)
    ssd = {k: v.to(dtype) for k, v in tiny_weights(False, meta["seed_s"], scfg).items()}
    tsd = {k: v.to(dtype) for k, v in tiny_weights(True, meta["seed_t"], tcfg).items()} if kind != "bd" else None
    tv, tp, tl = frozen(kind, phase)
    for k, v in ssd.items():
        train = (tl if k.startswith("language_model") else tp if (k.startswith("multi_modal") or k == "image_newline")
                 else tv)
        v.requires_grad_(train)
    b = batch(meta)
    for k in ("rgb_pixel_values", "depth_pixel_values"):
        b[k] = b[k].to(dtype)
    student = OracleLlava(ssd, scfg)
    teacher = OracleLlava(tsd, tcfg) if tsd else None
    total, aux = kd_step_losses(kind, teacher, student, b, phase=phase)
    total.float().backward()
    grads = {k: v.grad for k, v in ssd.items() if v.grad is not None and k != "language_model.lm_head.weight"}
    if with_logits:
        return float(total.detach()), grads, aux["s_logits"].detach()
    return float(total.detach()), grads


def grad_total_norm(grads) -> float:
    return math.sqrt(sum(float(g.double().pow(2).sum()) for g in grads.values()))
