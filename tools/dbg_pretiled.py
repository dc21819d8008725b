"""Debug: where the pre-tiled GEMM and v8 differ (epilogue variants) on one shape."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import ops  # noqa: E402
from test_gemm_gpu import _rand  # noqa: E402

dev = torch.device("cuda:0")
M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (1000, 1048, 600)
a = _rand(M, K, dev=dev, seed=401)
w = _rand(N, K, dev=dev, seed=402, scale=0.05)
wt = ops.pretile_b(w)
bias = _rand(N, dev=dev, seed=403)
res = _rand(M, N, dev=dev, seed=404)
for name, kw in [("plain", {}), ("f32", dict(out_dtype=torch.float32)), ("bias", dict(bias=bias)),
                 ("gelu", dict(act="gelu_tanh")), ("res", dict(residual=res)),
                 ("bias+gelu+res", dict(bias=bias, act="gelu_tanh", residual=res))]:
    x0 = ops.gemm(a, w, b_pretiled=wt, split_k=1, **kw)
    x1 = ops.gemm(a, w, variant=24, split_k=1, **kw)
    d = (x0.float() - x1.float()).abs()
    bad = (d > 0).nonzero()
    print(name, "ndiff", bad.shape[0], "max", d.max().item(),
          "rows", sorted(set(bad[:, 0].tolist()))[:8], "cols", sorted(set(bad[:, 1].tolist()))[:8], flush=True)
print("plan v24", ops.gemm_plan(a, w, variant=24, split_k=1), "plan v24 gelu", ops.gemm_plan(a, w, variant=24, split_k=1, act="gelu_tanh", bias=bias, residual=res))
