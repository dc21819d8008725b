"""How far the fp8 teacher's logits drift from the bf16 teacher's as depth grows (real
widths, random-init N(0, 0.02) weights, one 336x336 sample, L = 1536).

    python tools/fp8_depth_study.py [--depths 1,2,4,8,16,28] [--out profiles/r02/fp8_depth.json]

For each depth d the teacher has d Qwen2 layers and min(d, 26) SigLIP layers; the same
weights run once through the bf16 linears and once through the fp8 linears. Reported: the
teacher-logit rel-L2 / cosine and the last hidden state's rel-L2. GPU only."""
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
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (TEACHER_7B,
                                                                                                   LlavaOnevisionModel)
    dev = torch.device("cuda:0")
    b = synthetic_batch(1, dev, L=1536, seed=0)
    rows = []
    for d in (int(x) for x in a.depths.split(",")):
        cfg = replace(TEACHER_7B, vision=replace(TEACHER_7B.vision, layers=min(d, 26)),
                      text=replace(TEACHER_7B.text, layers=d))
        t = LlavaOnevisionModel(cfg, dev, trainable=False, seed=1)
        out = {}
        for name in ("bf16", "fp8"):
            if name == "fp8":
                t.enable_fp8()
            with torch.no_grad():
                f = t.forward(b["rgb_input_ids"], b["rgb_pixel_values"], b["image_sizes"], want_logits=True)
            torch.cuda.synchronize()
            out[name] = (f["hn"].float(), f["logits"].float())
        (hb, lb), (hf, lf) = out["bf16"], out["fp8"]
        r = dict(depth=d, logits_rel_l2=float((lf - lb).norm() / lb.norm()),
                 logits_cosine=float((lf * lb).sum() / (lf.norm() * lb.norm())),
                 hidden_rel_l2=float((hf - hb).norm() / hb.norm()),
                 argmax_agree=float((lf.argmax(-1) == lb.argmax(-1)).float().mean()))
        print(json.dumps(r), flush=True)
        rows.append(r)
        del t, out, hb, lb, hf, lf
        torch.cuda.empty_cache()
    if a.out:
        Path(a.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
