"""tune_gemm.py in the step's cache state: every (kernel/tile x split-K) candidate of the KD step's
GEMM shapes timed as single calls with operand B COLD (a 1 GiB write before each call evicts the
256 MB Infinity Cache and the L2s: weights in the forward and dgrad, saved activations in wgrad
are read a whole step after their last use) and operand A WARM (re-written just before, as its
producing kernel leaves it); median of --iters calls.  Same jsonl rows as tune_gemm.py, so
tools/fit_plan.py fits gemm.hip:plan_gemm to it.
    python tools/tune_gemm_cold.py tools/step_shapes_c1.json [top] [--iters 6]"""
import json
import os
import re
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
args = [x for x in sys.argv[1:] if not x.startswith("--")]
iters = 6
for i, x in enumerate(sys.argv):
    if x == "--iters":
        iters = int(sys.argv[i + 1])
src = args[0] if args else "tools/step_shapes_c1.json"
top = int(args[1]) if len(args) > 1 else 60
shapes = [r["shape"] for r in json.load(open(src))[:top]]
junk = torch.empty(1 << 28, dtype=torch.float32, device=dev)


def cold_time(f, a):
    ts = []
    for _ in range(iters):
        junk.fill_(1.0)
        a.mul_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


g = torch.Generator(device=dev).manual_seed(0)
for sh in shapes:
    if os.environ.get("TUNE_MATCH") and not re.search(os.environ["TUNE_MATCH"], sh):
        continue
    parts = sh.split(":")
    kind, (M, N, K) = parts[0], map(int, parts[1].split("x"))
    if kind not in ("gemm_kk", "gemm_kn", "gemm_nn"):
        continue   # the fused SwiGLU / dact builds have one kernel each
    f32 = parts[2] == "f32"
    acc = len(parts) > 3
    la, lb = kind[5], kind[6]
    a = torch.randn(K, M, device=dev, generator=g).bfloat16().t() if la == "n" else \
        torch.randn(M, K, device=dev, generator=g).bfloat16()
    b = torch.randn(K, N, device=dev, generator=g).bfloat16().t() if lb == "n" else \
        torch.randn(N, K, device=dev, generator=g).bfloat16()
    out = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    fl = 2.0 * M * N * K
    ops.gemm(a, b, out=out, accumulate=acc)
    auto = cold_time(lambda: ops.gemm(a, b, out=out, accumulate=acc), a)
    res = {}
    VARS = tuple(int(v) for v in os.environ.get("TUNE_VARS", "5,6,7,16").split(","))
    for var in VARS:
        for sk in (1, 2, 3, 4, 6, 8, 12, 16):
            if sk > 1 and (var == 1 or (K // 32) // sk < 4):
                continue
            if sk > 1 and sk * M * N * 4 > ops.GEMM_SPLITK_WS:
                continue
            f = lambda: ops.gemm(a, b, out=out, accumulate=acc, variant=var, split_k=sk)
            f()
            res[(var, sk)] = cold_time(f, a)
    best = min(res, key=res.get)
    row = dict(shape=sh, auto_ms=round(auto, 4), auto_tf=round(fl / auto / 1e9, 1), best=list(best),
               best_ms=round(res[best], 4), best_tf=round(fl / res[best] / 1e9, 1),
               s1={v: round(res[(v, 1)], 4) for v in VARS},
               all={f"{v}/{s}": round(t, 4) for (v, s), t in sorted(res.items())}, state="B cold, A warm")
    print(json.dumps(row), flush=True)
