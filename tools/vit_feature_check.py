"""Diagnostic: the HIP vision tower's post-LN hook features (student and teacher) against the
CPU fp32 oracle on a tiny end-to-end fixture, with the student's residual streams in fp32
and in bf16.  GPU only.    python tools/vit_feature_check.py [fixture]"""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests" / "golden"))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "dt1"
    from model_fixtures import batch, load, tiny_weights
    from oracle.model import OracleLlava
    from oracle import kd_losses as KL
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (
        LlavaOnevisionModel, tiny_config)
    meta, exp = load(name)
    dev = torch.device("cuda:0")
    bc = batch(meta)
    for who, seed, teacher in (("student", meta["seed_s"], False), ("teacher", meta["seed_t"], True)):
        cfg = tiny_config(teacher)
        o = OracleLlava(tiny_weights(teacher, seed), cfg)
        key = "rgb" if teacher else "depth"
        with torch.no_grad():
            _, post = o(bc[f"{key}_input_ids"], bc[f"{key}_pixel_values"].float(), bc["image_sizes"])
        ref = KL.pooled_features(post)
        for rf in ((False, False), (True, True)):
            m = LlavaOnevisionModel(cfg, dev, trainable=not teacher, seed=seed, cpu_rng=True)
            m.set_residual_f32(*rf)
            b = batch(meta, dev)
            with torch.no_grad():
                f = m.forward(b[f"{key}_input_ids"], b[f"{key}_pixel_values"], b["image_sizes"], want_post_ln=True)
            torch.cuda.synchronize()
            got_post = f["post_ln"].float().cpu().view(post.shape)
            got = KL.pooled_features(got_post)
            rel_post = float((got_post - post).norm() / post.norm())
            rel = float((got - ref).norm() / ref.norm())
            # the tile-to-tile differences NT-Xent feeds on
            d_ref = ref - ref.mean(0, keepdim=True)
            d_got = got - got.mean(0, keepdim=True)
            rel_d = float((d_got - d_ref).norm() / d_ref.norm())
            print(f"{who} residual_f32={rf}: post-LN rel {rel_post:.3e}  pooled rel {rel:.3e}  "
                  f"pooled minus mean rel {rel_d:.3e}  (|d_ref|/|ref| {float(d_ref.norm() / ref.norm()):.3e})",
                  flush=True)
            ntx = float(KL.nt_xent(got, ref))
            print(f"   nt_xent(got, oracle) {ntx:.6f}", flush=True)


if __name__ == "__main__":
    main()
