"""Generate golden fixtures from the REFERENCE's own code (run in the dev container only).

    python tests/golden/make_golden.py [--only NAME]

Imports the reference modules from /root/reference with a 5-line `pytorch_lightning`
stub (the package is not installed), binds their loss methods to bare
instances carrying the hard-coded hyper-parameters (DT:67-71, LB:73-75, FB:72-74),
and records their outputs on seeded inputs (tests/golden/inputs.py).  Only outputs
are committed (tests/golden/*.npz / kat.json); the reference never leaves this
container, in any form.  The student CE is transformers' ForCausalLMLoss, which is
what LlavaOnevisionForConditionalGeneration.forward computes for `labels=` (the
reference reads it as `student_outputs.loss`, DT:240).
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import inputs as I  # noqa: E402

REF = Path("/root/reference")
DT_PATH = REF / "distillation/knowledge_distillation7b_double_trouble/phase1/OnlineKnowledgeDistillationLLavaOneVision.py"
LB_PATH = REF / "distillation/knowledge_distillation7b_logit_based/OnlineKnowledgeDistillationLLavaOneVision.py"
FB_PATH = REF / "distillation/knowledge_distillation7b_feature_based/OnlineKnowledgeDistillationLLavaOneVision.py"


def _install_stub():
    d = Path(tempfile.mkdtemp(prefix="plstub_")) / "pytorch_lightning"
    d.mkdir(parents=True)
    (d / "__init__.py").write_text(
        "import torch.nn as nn\nclass LightningModule(nn.Module):\n    def log(self, *a, **k):\n        pass\n")
    sys.path.insert(0, str(d.parent))
    sys.path.insert(0, str(REF))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m.OnlineKnowledgeDistillationLLavaOneVision


BD_PATH = REF / "distillation/baseline_depth/LLavaOneVisionModule.py"


def _load_bd():
    spec = importlib.util.spec_from_file_location("ref_bd", BD_PATH)
    m = importlib.util.module_from_spec(spec)
    sys.modules["ref_bd"] = m
    spec.loader.exec_module(m)
    return m.LlavaOnevisionModule


def _bare(cls, **attrs):
    obj = cls.__new__(cls)
    torch.nn.Module.__init__(obj)
    for k, v in attrs.items():
        setattr(obj, k, v)
    return obj


def ref_modules():
    _install_stub()
    DT, LB, FB = _load("ref_dt", DT_PATH), _load("ref_lb", LB_PATH), _load("ref_fb", FB_PATH)
    dt = _bare(DT, T=0.8, gamma=0.8, soft_target_loss_weight=0.1, ce_loss_weight=0.5, phase=2)
    lb = _bare(LB, T=1, soft_target_loss_weight=0.5, ce_loss_weight=0.5)
    fb = _bare(FB, T=0.8, soft_target_loss_weight=0.1, ce_loss_weight=0.8)
    return dt, lb, fb


def hf_ce(logits, labels):
    from transformers.loss.loss_utils import ForCausalLMLoss
    return ForCausalLMLoss(logits, labels, vocab_size=logits.shape[-1])


CASES = {
    # name: recipe
    "loca_dt_T08_B1_L1536": dict(variant="loca", module="dt", B=1, L=1536, seed=11, labels="layout"),
    "loca_lb_T1_B1_L1536": dict(variant="loca", module="lb", B=1, L=1536, seed=12, labels="layout"),
    "loca_lb_T1_B2_L768_rand": dict(variant="loca", module="lb", B=2, L=768, seed=13, labels="random"),
    "loca_dt3_T08_B4_L128_rand": dict(variant="loca", module="dt3", B=4, L=128, seed=17, labels="random"),
    "kl_dt1_T08_B2_L512": dict(variant="kl", module="dt1", B=2, L=512, seed=14, labels="layout"),
    "kllt_fb_T08_B2_L512": dict(variant="kllt", module="fb", B=2, L=512, seed=15, labels="layout"),
    "ce_bd_B2_L512_pad": dict(variant="ce", module="bd", B=2, L=512, seed=16, labels="pad"),
}


def make_labels(rec):
    B, L, seed = rec["B"], rec["L"], rec["seed"]
    if rec["labels"] == "layout":
        n_img = min(I.N_IMAGE_TOKENS_336, L - 40)
        return I.token_ids(B, L, seed=seed, n_image=n_img)
    if rec["labels"] == "random":
        g = torch.Generator().manual_seed(seed + 1000)
        # few distinct ids so the global overrides collide often (KAT 1)
        return torch.randint(0, 64, (B, L), generator=g) * 2371
    if rec["labels"] == "pad":
        ids = I.token_ids(B, L, seed=seed, n_image=min(I.N_IMAGE_TOKENS_336, L - 40))
        ids[1, L - 100:] = -100  # right-padding of the second sample (DM:145-146)
        return ids
    raise ValueError(rec["labels"])


def case_inputs(rec):
    labels = make_labels(rec)
    t, s = I.kd_logits(rec["B"], rec["L"], rec["seed"], labels.clamp(min=0))
    return t, s, labels


def run_case(name, rec, dt, lb, fb):
    t, s, labels = case_inputs(rec)
    s = s.clone().requires_grad_(True)
    V = s.shape[-1]
    ce = hf_ce(s, labels)
    with torch.no_grad():
        tce = hf_ce(t, labels)
    var, mod = rec["variant"], rec["module"]
    if var == "loca":
        m = lb if mod == "lb" else dt
        kd = m.compute_loca_loss(t, s, torch.zeros(()), labels)          # loca term only
        loca_plus_ce = m.compute_loca_loss(t, s, ce, labels)            # DT:194 / LB:261
        if mod == "dt3":   # DT:257-260
            total = dt.gamma * loca_plus_ce + (1 - dt.gamma) * ce
        else:
            total = loca_plus_ce
        kd_weight, ce_weight, T = (0.8 if mod == "dt3" else 1.0), 1.0, float(m.T)
    elif var == "kl":
        outs = types.SimpleNamespace(logits=s, loss=ce)
        zero = lambda *a, **k: torch.zeros(())  # isolate the KL term of compute_vision_loss
        dt.contrastive_loss = zero
        weighted = dt.compute_vision_loss(None, None, t, outs)           # 0.1 * KL * T^2
        del dt.contrastive_loss
        kd = weighted / dt.soft_target_loss_weight
        total = weighted
        kd_weight, ce_weight, T = dt.soft_target_loss_weight, 0.0, float(dt.T)
    elif var == "kllt":
        outs0 = types.SimpleNamespace(logits=s, loss=torch.zeros(()))
        weighted = fb.compute_loss(t, outs0, torch.zeros(()))             # 0.1 * KLq * T^2
        kd = weighted / fb.soft_target_loss_weight
        outs = types.SimpleNamespace(logits=s, loss=ce)
        total = fb.compute_loss(t, outs, torch.zeros(()))                 # + 0.8 CE (ctr = 0)
        kd_weight, ce_weight, T = fb.soft_target_loss_weight, fb.ce_loss_weight, float(fb.T)
    elif var == "ce":
        kd = torch.zeros(())
        total = ce
        kd_weight, ce_weight, T = 0.0, 1.0, 1.0
    else:
        raise ValueError(var)
    if var != "ce":   # gradient of the weighted KD term alone (it is ~1e-6 of the CE's)
        gk = torch.autograd.grad(kd * kd_weight, s, retain_graph=True)[0].detach().reshape(-1, V)
    else:
        gk = torch.zeros(s.shape).reshape(-1, V)
    total.backward()
    g = s.grad.detach().reshape(-1, V)
    R = g.shape[0]
    gen = torch.Generator().manual_seed(rec["seed"] + 7)
    rows_idx = torch.tensor([0, R // 2, R - 1])
    samp = torch.stack([torch.randint(0, R, (4096,), generator=gen),
                        torch.randint(0, V, (4096,), generator=gen)], 1)
    out = dict(
        gk_rowsum=gk.sum(1).double().numpy(), gk_rowabs=gk.abs().sum(1).double().numpy(),
        gk_rows=gk[rows_idx].numpy().astype(np.float32),
        gk_samp_val=gk[samp[:, 0], samp[:, 1]].numpy().astype(np.float32),
        kd_term=np.float64(kd.item()), ce=np.float64(ce.item()), teacher_ce=np.float64(tce.item()),
        total=np.float64(total.item()),
        g_rowsum=g.sum(1).double().numpy(), g_rowabs=g.abs().sum(1).double().numpy(),
        g_rows_idx=rows_idx.numpy(), g_rows=g[rows_idx].numpy().astype(np.float32),
        g_samp_idx=samp.numpy(), g_samp_val=g[samp[:, 0], samp[:, 1]].numpy().astype(np.float32),
        t_ck=np.array(I.checksum(t)), s_ck=np.array(I.checksum(s)), labels_ck=np.array(I.checksum(labels)),
    )
    meta = dict(rec, name=name, kd_weight=kd_weight, ce_weight=ce_weight, T=T, alpha=0.8,
                V_s=V, V_t=t.shape[-1])
    np.savez_compressed(HERE / f"kd_{name}.npz", meta=json.dumps(meta), **out)
    print(f"{name}: kd={kd.item():.8g} ce={ce.item():.8g} tce={tce.item():.8g} total={total.item():.8g}")


def make_kats(dt, lb, fb):
    """Known-answer tests of SURVEY §4, recorded from the reference."""
    kat = {}
    # KAT 1: small LoCa with duplicate labels -> record inputs and outputs
    g = torch.Generator().manual_seed(5)
    B, L, V = 2, 5, 16
    t = torch.randn(B, L, V + 3, generator=g) * 2
    s = (torch.randn(B, L, V, generator=g) * 2).requires_grad_(True)
    labels = torch.tensor([[3, 7, 3, 1, 7], [7, 0, 3, 9, 1]])
    loss = lb.compute_loca_loss(t, s, torch.zeros(()), labels)
    loss.backward()
    # q matrix as the reference builds it (DT:183-185) via a capture of F.kl_div's target
    import torch.nn.functional as Fm
    captured = {}
    orig = Fm.kl_div

    def cap(inp, target, **kw):
        captured["q"] = target.detach().clone()
        return orig(inp, target, **kw)
    ref_F = sys.modules["ref_lb"].F
    ref_F.kl_div = cap
    try:
        lb.compute_loca_loss(t, s.detach(), torch.zeros(()), labels)
    finally:
        ref_F.kl_div = orig
    kat["kat1"] = dict(t=t.tolist(), s=s.detach().tolist(), labels=labels.tolist(), T=1.0,
                       loss=loss.item(), grad=s.grad.tolist(), q=captured["q"].tolist())
    # KAT 2: -100 crashes LoCa
    try:
        lab2 = labels.clone(); lab2[0, 0] = -100
        lb.compute_loca_loss(t, s.detach(), torch.zeros(()), lab2)
        kat["kat2"] = dict(raised=False)
    except (RuntimeError, IndexError) as e:
        kat["kat2"] = dict(raised=True, type=type(e).__name__)
    # KAT 6: topk(2) tie order of torch CPU
    v = torch.tensor([[.1, .5, .3, .5, .5, .2]])
    kat["kat6"] = dict(values=v.tolist(), topk2_indices=torch.topk(v, 2, dim=-1).indices.tolist())
    # KAT 5: clamp zeroes the gradient where p_S < 1e-8
    s5 = torch.zeros(1, 2, 8)
    s5[..., 0] = 30.0                              # others: p ~ exp(-30) < 1e-8
    s5.requires_grad_(True)
    t5 = torch.randn(1, 2, 8, generator=g)
    l5 = lb.compute_loca_loss(t5, s5, torch.zeros(()), torch.tensor([[1, 2]]))
    l5.backward()
    kat["kat5"] = dict(t=t5.tolist(), s=s5.detach().tolist(), labels=[[1, 2]], loss=l5.item(),
                       grad=s5.grad.tolist())
    # KAT 9: image-token counts of the anyres pack for 336x336 and 480x640 (H, W)
    from transformers.models.llava_onevision.modeling_llava_onevision import image_size_to_num_patches
    from transformers import LlavaOnevisionConfig
    cfg = LlavaOnevisionConfig()
    kat["kat9"] = {}
    for hw in ([336, 336], [480, 640]):
        n_p = image_size_to_num_patches(hw, cfg.image_grid_pinpoints, cfg.vision_config.image_size)
        kat["kat9"][f"{hw[0]}x{hw[1]}"] = dict(num_patches=n_p, num_tokens=_hf_pack_tokens(cfg, hw, n_p))
    # NT-Xent (DT:393-416) on pooled features (DT:243-248) of 2B = 4 tiles
    sf, tf = I.features(4, 1152, seed=21)
    sf = sf.requires_grad_(True)
    sp = torch.nn.functional.normalize(sf.mean(dim=1), p=2, dim=-1)
    tp = torch.nn.functional.normalize(tf.mean(dim=1), p=2, dim=-1)
    ctr = dt.contrastive_loss(sp, tp)
    ctr.backward()
    gsf = sf.grad
    kat["ntxent"] = dict(seed=21, n=4, dim=1152, tokens=729, loss=ctr.item(),
                         grad_sum=float(gsf.double().sum()), grad_abs=float(gsf.double().abs().sum()),
                         grad_row0=gsf[0, 0, :16].tolist(),
                         s_ck=I.checksum(sf.detach()), t_ck=I.checksum(tf))
    (HERE / "kat.json").write_text(json.dumps(kat))
    print("KATs:", {k: (v if k in ("kat2", "kat6") else "...") for k, v in kat.items()})


def _hf_pack_tokens(cfg, hw, n_p):
    """Run HF's own pack_image_features on dummy features to count image tokens."""
    from transformers.models.llava_onevision.modeling_llava_onevision import LlavaOnevisionModel
    m = LlavaOnevisionModel.__new__(LlavaOnevisionModel)
    m.config = cfg
    feats = [torch.zeros(n_p, 729, 4)]
    packed, lens = LlavaOnevisionModel.pack_image_features(m, feats, torch.tensor([hw]), image_newline=torch.zeros(4))
    return int(lens[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--kats", action="store_true")
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    dt, lb, fb = ref_modules()
    if a.kats or a.only is None:
        make_kats(dt, lb, fb)
    for name, rec in CASES.items():
        if a.only and a.only != name:
            continue
        if a.kats and a.only is None:
            continue
        run_case(name, rec, dt, lb, fb)


if __name__ == "__main__":
    main()
