"""Where the error of the NT-Xent-only SigLIP post_layernorm.bias gradient comes from (real_dt1,
real_fb: the reference's fp32 forward at the real widths, 2 layers per tower).

    python tools/ntx_bias_study.py [kind ...]

post_layernorm's output feeds only the hook (DT:100-121 -> mean over the 729 patches -> NT-Xent,
DT:243-248, :393-416; the projector reads hidden_states[-1], before post_layernorm), so
d/d(post_layernorm.bias) = sum over tiles of d(loss)/d(pooled tile feature).  From the HIP
step's own post-LN hook outputs (bf16, last_post) this computes in fp64:
  given_fwd    the exact bias gradient for HIP's features (backward correctness)
  given_fwd_b  the same with d(pooled)/729 rounded to bf16 per element (what the round-4 bf16 dpost
               held: HIP matched it to 1e-5, i.e. that rounding WAS the error; since ABI 7 the hook
               gradient reaches the LayerNorm backward in fp32 and HIP matches given_fwd)
and compares HIP's bias gradient and the reference's (fixture, fp32) against both, plus the
tiles' pooled-feature cosines (the cancellation that amplifies any feature error).  GPU only.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "tests" / "golden"))


def study(name, dev):
    import numpy as np
    import torch
    from step_parity import hip_grad, run_step
    from model_fixtures import EVERY_KIND
    m, meta, exp, loss = run_step(name, dev)
    kind, phase = EVERY_KIND[name]
    ctr_w = m._loss_spec()[4]
    sp, tp = m.last_post
    NP = m.student_model.cfg.vision.n_patches
    ps = sp.double().cpu().view(-1, NP, sp.shape[-1]).mean(1).requires_grad_(True)
    pt = tp.double().cpu().view(-1, NP, tp.shape[-1]).mean(1)
    from oracle import kd_losses as O
    ntx = O.nt_xent(O.l2_normalize(ps), O.l2_normalize(pt)) * ctr_w
    g, = torch.autograd.grad(ntx, ps)
    exact = g.sum(0)
    rounded = (NP * (g / NP).to(torch.bfloat16).double()).sum(0)
    names = [str(n) for n in exp["grad_names"]]
    n = "vision_tower.vision_model.post_layernorm.bias"
    i = names.index(n)
    ref = torch.from_numpy(np.asarray(exp["grad_samples"][i][:exact.numel()])).double()
    hip = hip_grad(m.student_model.P, n).double().cpu().reshape(-1)

    def cmp(a, b):
        return dict(rel_err=float((a - b).norm() / b.norm()), norm_rel=float(a.norm() / b.norm() - 1),
                    cos=float(a @ b / (a.norm() * b.norm())))
    f = torch.nn.functional.normalize(ps.detach(), dim=-1)
    cosm = (f @ f.t()).numpy()
    out = dict(ntx_weight=ctr_w, tiles=int(ps.shape[0]), ref_norm=float(ref.norm()), exact_norm=float(exact.norm()),
               per_tile_grad_norm=[float(v) for v in g.norm(dim=-1)],
               cancellation=float(exact.norm() / g.norm(dim=-1).sum()),
               student_tile_cos=cosm.tolist(),
               hip_vs_given_fwd=cmp(hip, exact), hip_vs_given_fwd_bf16dpost=cmp(hip, rounded),
               given_fwd_vs_ref=cmp(exact, ref), hip_vs_ref=cmp(hip, ref))
    del m
    torch.cuda.empty_cache()
    return out


def main():
    import torch
    kinds = sys.argv[1:] or ["real_dt1", "real_fb"]
    rep = {k: study(k, torch.device("cuda:0")) for k in kinds}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
