"""Time the student generate() (evaluate_onevision.py:185-195 settings) on the real 0.5B student:
prefill of one 336x336 prompt (L = 1536) + 32 greedy decode steps with the KV cache.
    python tools/bench_generate.py"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.data import synthetic_batch  # noqa
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.generation import generate  # noqa
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (  # noqa
    STUDENT_05B, LlavaOnevisionModel)

dev = torch.device("cuda:0")
model = LlavaOnevisionModel(STUDENT_05B, dev, seed=2)
b = synthetic_batch(1, dev, L=1536, seed=0)
kw = dict(repetition_penalty=1.2, no_repeat_ngram_size=2, eos_token_id=())


def timed(n_new):
    generate(model, b["depth_input_ids"], b["depth_pixel_values"], b["image_sizes"], max_new_tokens=n_new, **kw)
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        t0 = time.perf_counter()
        generate(model, b["depth_input_ids"], b["depth_pixel_values"], b["image_sizes"], max_new_tokens=n_new, **kw)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


t32, t96 = timed(32), timed(96)
t0 = time.perf_counter()
model.forward(b["depth_input_ids"], b["depth_pixel_values"], b["image_sizes"])
torch.cuda.synchronize()
pre = time.perf_counter() - t0
print(f"generate 0.5B student, 336x336 prompt (L=1536) + 32 tokens: {t32 * 1e3:.1f} ms per call "
      f"(prefill forward {pre * 1e3:.1f} ms); graph-replayed decode step {(t96 - t32) / 64 * 1e3:.3f} ms/token "
      f"(marginal cost from 32 -> 96 new tokens)")
