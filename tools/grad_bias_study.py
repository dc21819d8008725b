"""Where does the bf16 gradient-norm bias come from?  

Runs the CPU oracle step of a tiny end-to-end fixture (tests/golden/model_<kind>.npz) in
fp32 and in bf16 and prints, per parameter group, the gradient norm of each and the
relative difference, sorted by each group's share of the total-norm difference
(d||g||^2 = sum over groups of d||g_i||^2).

    python tools/grad_bias_study.py lb [dt1 ...]
"""
from __future__ import annotations

import math
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests" / "golden"))

from model_fixtures import oracle_grads  # noqa: E402


def group(name: str) -> str:
    for tag in ("embed_tokens", "lm_head", "norm.weight", "patch_embedding", "position_embedding",
                "post_layernorm", "multi_modal_projector", "image_newline"):
        if tag in name:
            return name
    parts = name.split(".")
    return ".".join(p for p in parts if not p.isdigit())


def main(kinds):
    for kind in kinds:
        _, g32 = oracle_grads(kind)
        _, g16 = oracle_grads(kind, torch.bfloat16)
        n32 = math.sqrt(sum(float(g.double().pow(2).sum()) for g in g32.values()))
        n16 = math.sqrt(sum(float(g.double().pow(2).sum()) for g in g16.values()))
        print(f"== {kind}: total |g| fp32 {n32:.6g} bf16 {n16:.6g} rel {n16 / n32 - 1:+.3e}")
        rows = {}
        for k, g in g32.items():
            a = float(g.double().pow(2).sum())
            b = float(g16[k].double().pow(2).sum())
            c = float((g.double() - g16[k].double()).pow(2).sum())
            r = rows.setdefault(group(k), [0.0, 0.0, 0.0])
            r[0] += a; r[1] += b; r[2] += c
        dsq = n16 ** 2 - n32 ** 2
        for k, (a, b, c) in sorted(rows.items(), key=lambda kv: -abs(kv[1][1] - kv[1][0])):
            if a == 0:
                continue
            print(f"  {k:70s} |g| {math.sqrt(a):10.4g}  rel {math.sqrt(b / a) - 1:+.3e}  "
                  f"share {(b - a) / dsq:+.3f}  |d|/|g| {math.sqrt(c / a):.3e}")


if __name__ == "__main__":
    main(sys.argv[1:] or ["lb"])
