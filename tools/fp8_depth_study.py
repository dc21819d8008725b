"""How far the fp8 teacher's logits drift from the bf16 teacher's as depth grows (real
widths, random-init N(0, 0.02) weights, one 336x336 sample, L = 1536).

    python tools/fp8_depth_study.py [--depths 1,2,4,8,16,28] [--families all,lm,lm_body,lm_mlp]
                                    [--batch 1] [--out profiles/r03/fp8_depth.json]

For each depth d the teacher has d Qwen2 layers and min(d, 26) SigLIP layers; the same
weights run once through the bf16 linears and once per fp8 policy (which linear families run
on the fp8 GEMM, modeling.FP8_FAMILIES). Reported: the teacher-logit rel-L2 / cosine, the
last hidden state's rel-L2 and the forward time of each (HIP events). GPU only."""
from __future__ import annotations

import argparse
import json
import sys
from dataclasses import replace
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depths", default="1,2,4,8,16,28")
    ap.add_argument("--families", default="all", help="comma list of modeling.FP8_FAMILIES policies")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (TEACHER_7B,
                                                                                                   LlavaOnevisionModel)
    dev = torch.device("cuda:0")
    b = synthetic_batch(a.batch, dev, L=1536, seed=0)
    rows = []

    def run(t):
        with torch.no_grad():
            f = t.forward(b["rgb_input_ids"], b["rgb_pixel_values"], b["image_sizes"], want_logits=True)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            t.forward(b["rgb_input_ids"], b["rgb_pixel_values"], b["image_sizes"], want_logits=True)
            ev[1].record()
        torch.cuda.synchronize()
        return f["hn"].float(), f["logits"].float(), ev[0].elapsed_time(ev[1])

    for d in (int(x) for x in a.depths.split(",")):
        cfg = replace(TEACHER_7B, vision=replace(TEACHER_7B.vision, layers=min(d, 26)),
                      text=replace(TEACHER_7B.text, layers=d))
        t = LlavaOnevisionModel(cfg, dev, trainable=False, seed=1)
        hb, lb, ms_b = run(t)
        for fam in a.families.split(","):
            t.enable_fp8(fam)
            hf, lf, ms_f = run(t)
            t.disable_fp8()
            r = dict(depth=d, families=fam, logits_rel_l2=float((lf - lb).norm() / lb.norm()),
                     logits_cosine=float((lf * lb).sum() / (lf.norm() * lb.norm())),
                     hidden_rel_l2=float((hf - hb).norm() / hb.norm()),
                     argmax_agree=float((lf.argmax(-1) == lb.argmax(-1)).float().mean()),
                     fwd_ms_fp8=round(ms_f, 2), fwd_ms_bf16=round(ms_b, 2), batch=a.batch)
            print(json.dumps(r), flush=True)
            rows.append(r)
            del hf, lf
        del t, hb, lb
        torch.cuda.empty_cache()
    if a.out:
        Path(a.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
