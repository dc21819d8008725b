"""The bf16 floor of the end-to-end fixtures (dev container, CPU).

    python tests/golden/make_bf16_floor.py [kind ...]

For every tiny end-to-end fixture (tests/golden/model_*.npz, the reference's own forward in
fp32) the CPU oracle (oracle/model.py, pinned to those fixtures in fp32) is run again with
bf16 weights and activations (torch autograd on the CPU): how far a plain bf16 run of the
reference's arithmetic lands from the fp32 reference.  Recorded per kind, in
tests/golden/bf16_floor.json: the step's total loss, the gradient's total norm, and on the fixture's sampled
student-logit rows the fraction of elements within the north-star |d| <= 1e-4 + 1e-3 |ref|
and the largest |d|; per parameter, the gradient norm's relative miss and the cosine to the
reference gradient (param_floor).  tests/test_kd_step_gpu.py holds the HIP path (bf16 storage, fp32
accumulation) to this floor where the north-star tolerance is below bf16 resolution (raw
logits of magnitude ~0.2 have a bf16 half-ulp of ~5e-4 > 1e-4 + 1e-3 |ref|).
"""
from __future__ import annotations

import json
import math
import os
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.path.insert(0, str(HERE))

from model_fixtures import EVERY_KIND, grad_sample_index, grad_total_norm, load, oracle_grads  # noqa: E402

OUT = HERE / "bf16_floor.json"
ATOL, RTOL = 1e-4, 1e-3


def param_floor(name, exp, g):
    """Per parameter: how far the plain-bf16 gradient lands from the reference's —
    norm_rel = | |g_bf16| / |g_ref| - 1 | against the reference's recorded norms, and the
    cosine against the reference gradient: the fp32 oracle's full vectors for the tiny
    fixtures (pinned to the reference, tests/test_oracle_model.py), the reference's own
    sampled entries for the real-width ones (model_fixtures.grad_sample_index)."""
    names = [str(n) for n in exp["grad_names"]]
    out = {}
    ref32 = None
    if "grad_samples" not in exp:
        _, ref32 = oracle_grads(name)
    for i, n in enumerate(names):
        gb = g[n].double().reshape(-1)
        rn = float(exp["grad_norms"][i])
        if "grad_samples" in exp:
            idx = grad_sample_index(n, gb.numel())
            a = gb[idx]
            b = torch.from_numpy(exp["grad_samples"][i][:idx.numel()]).double()
        else:
            a, b = gb, ref32[n].double().reshape(-1)
        cos = float((a @ b) / (a.norm() * b.norm() + 1e-300))
        out[n] = dict(norm_rel=abs(float(gb.norm()) / rn - 1) if rn > 0 else 0.0, cos=cos, ref_norm=rn)
    return out


def floor(name):
    _, exp = load(name)
    total, g, logits = oracle_grads(name, torch.bfloat16, with_logits=True)
    rows = exp["logit_rows"].tolist()
    st = int(exp["logit_col_stride"])
    got = logits[:, rows, ::st].float().numpy()
    ref = exp["s_logit_rows"]
    err = np.abs(got - ref)
    del logits
    return dict(total=float(total), ref_total=float(exp["total"]),
                grad_total_norm=grad_total_norm(g), ref_grad_total_norm=float(exp["grad_total_norm"]),
                logit_frac_within_north_star=float((err <= ATOL + RTOL * np.abs(ref)).mean()),
                logit_max_abs=float(err.max()), logit_rms_ref=float(math.sqrt(float((ref ** 2).mean()))),
                params=param_floor(name, exp, g))


def main():
    torch.set_num_threads(os.cpu_count())
    res = json.loads(OUT.read_text()) if OUT.exists() else {}
    for name in (sys.argv[1:] or list(EVERY_KIND)):
        res[name] = floor(name)
        print(name, res[name], flush=True)
        OUT.write_text(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
