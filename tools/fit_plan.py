"""Fit gemm.hip:plan_gemm's cost model to a tune_gemm.py sweep and report how close the
model's picks come to the measured best, weighted by each shape's launches per step.
    python tools/fit_plan.py gemm_tune.jsonl [step_shapes.json]
Model (microseconds): waves x (k-steps per split x step[v,c] + fixed[v,c]) + split traffic / BW
(+ a fixed cost of the split's reduce launch),
v = kernel/tile (v3 256x256, 256x128, 128x256, v8), c = operand class (K-major x K-major, other)."""
import json
import math
import sys

import numpy as np
from scipy.optimize import least_squares

rows = [json.loads(l) for l in open(sys.argv[1])]
w = {r["shape"]: r["launches"] for r in json.load(open(sys.argv[2] if len(sys.argv) > 2 else "tools/step_shapes_c1.json"))}
VI = {5: 0, 6: 1, 7: 2, 16: 3, 20: 4}
NV = 5


def cd(a, b):
    return (a + b - 1) // b


def feats(shape, v, S):
    p = shape.split(":")
    M, N, K = map(int, p[1].split("x"))
    f32, acc = p[2] == "f32", len(p) > 3
    c = 0 if p[0] == "gemm_kk" else 1
    tiles = [cd(M, 256) * cd(N, 256), cd(M, 256) * cd(N, 128), cd(M, 128) * cd(N, 256), cd(M, 256) * cd(N, 256),
             cd(M, 256) * cd(N, 256)][v]
    nk = cd(K, 32)
    kcs = cd(nk, S)
    waves = cd(tiles * S, 256)
    out_b = M * N * ((4 if f32 else 2) * (2 if acc else 1))
    traffic = (S * M * N * 8 + out_b) if S > 1 else 0.0
    return c, waves, kcs, traffic


data = []
for r in rows:
    for key, ms in r["all"].items():
        v, S = map(int, key.split("/"))
        data.append((r["shape"], VI[v], S, ms * 1e3))


def pred(x, shape, v, S):
    c, waves, kcs, traffic = feats(shape, v, S)
    step, fixed = x[2 * (NV * c + v)], x[2 * (NV * c + v) + 1]
    return waves * (kcs * step + fixed) + traffic / (x[4 * NV] * 1e6) + (x[4 * NV + 1] if S > 1 else 0.0)


def resid(x):
    return [math.log(max(pred(x, s, v, S), 1e-3)) - math.log(t) for s, v, S, t in data]


x0 = np.array([0.8, 4.0] * (2 * NV) + [6.0, 2.0])
fit = least_squares(resid, x0, bounds=([0.05, 0.0] * (2 * NV) + [1.0, 0.0], [5.0, 50.0] * (2 * NV) + [20.0, 50.0]))
x = fit.x
print("step/fixed per class (kk, mn) x variant (v3 256x256, 256x128, 128x256, v8, v9); BW TB/s", round(x[4 * NV], 3),
      "; split launch us", round(x[4 * NV + 1], 3))
for c in range(2):
    print(" ", ["kk", "mn"][c], [(round(x[2 * (NV * c + v)], 4), round(x[2 * (NV * c + v) + 1], 3)) for v in range(NV)])
tot_best = tot_pick = 0.0
for r in rows:
    meas = {(VI[int(k.split("/")[0])], int(k.split("/")[1])): t * 1e3 for k, t in r["all"].items()}
    pick = min(meas, key=lambda vs: pred(x, r["shape"], *vs))
    best = min(meas.values())
    n = w.get(r["shape"], 1)
    tot_best += n * best
    tot_pick += n * meas[pick]
    if meas[pick] > 1.05 * best:
        print(f"  {r['shape']:40s} pick {pick} {meas[pick]:8.1f} us  best {best:8.1f} us")
print(f"per step: picks {tot_pick / 1e3:.1f} ms vs measured best {tot_best / 1e3:.1f} ms")
