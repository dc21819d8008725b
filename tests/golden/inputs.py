"""Deterministic synthetic inputs shared by the golden-fixture maker and the tests.

Everything is generated on the CPU with torch.Generator(seed) so the same values are
reproduced on the GPU box (same image, same torch) without shipping large tensors:
a fixture stores only the seed/shape recipe, input checksums and expected outputs.

Token layout (the 336x336 synthetic config):
  L = 24 text ids + 1485 image tokens (id 151646) + 27 text ids, text ids ~ U[0, 151643);
  labels = input_ids (no -100: sequences have equal length, DM:145-146).
"""
from __future__ import annotations

import torch

IMAGE_TOKEN_ID = 151646          # LlavaOnevisionConfig.image_token_index
TEXT_VOCAB = 151643              # text ids drawn below the special tokens
V_STUDENT = 151936               # Qwen2-0.5B vocab (student lm_head rows)
V_TEACHER = 152064               # Qwen2-7B vocab (teacher lm_head rows)
N_IMAGE_TOKENS_336 = 1485        # 729 base + 27*(27+1) grid tokens (SURVEY §4 KAT 9)


def token_ids(B: int, L: int = 1536, seed: int = 0, n_image: int = N_IMAGE_TOKENS_336,
              prefix: int = 24) -> torch.Tensor:
    """[B, L] int64: prefix text ids, n_image image tokens, then text ids."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, TEXT_VOCAB, (B, L), generator=g, dtype=torch.int64)
    if n_image:
        assert prefix + n_image <= L
        ids[:, prefix:prefix + n_image] = IMAGE_TOKEN_ID
    return ids


def _bf16(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).to(torch.float32)


def kd_logits(B: int, L: int, seed: int, labels: torch.Tensor, V_s: int = V_STUDENT,
              V_t: int = V_TEACHER, sigma_t: float = 2.0, sigma_s: float = 2.0,
              agree_frac: float = 0.5):
    """Teacher/student logits, bf16-representable fp32 tensors [B,L,V_t] / [B,L,V_s].

    The teacher's top-2 over [0, V_s) is made unique and tie-free (SURVEY §4 KAT 6):
    per row the top-1 is at the label for an `agree_frac` share of rows (else a random
    column) and sits 2.0 above the row max, the top-2 at another column 1.0 above.
    """
    g = torch.Generator().manual_seed(seed)
    t = _bf16(torch.randn(B, L, V_t, generator=g) * sigma_t)
    s = _bf16(torch.randn(B, L, V_s, generator=g) * sigma_s)
    R = B * L
    tf = t.view(R, V_t)
    rmax = tf[:, :V_s].amax(dim=1)
    p1 = torch.randint(0, V_s, (R,), generator=g)
    p2 = torch.randint(0, V_s, (R,), generator=g)
    agree = torch.rand(R, generator=g) < agree_frac
    lab = labels.reshape(-1)
    p1 = torch.where(agree & (lab >= 0) & (lab < V_s), lab, p1)
    p2 = torch.where(p2 == p1, (p2 + 1) % V_s, p2)
    ar = torch.arange(R)
    tf[ar, p1] = _bf16(rmax + 2.0)
    tf[ar, p2] = _bf16(rmax + 1.0)
    # verify uniqueness of the top-2 values (strictly above everything else)
    top = torch.topk(tf[:, :V_s], 3, dim=1).values
    assert bool((top[:, 0] > top[:, 1]).all() and (top[:, 1] > top[:, 2]).all()), "ties in top-3"
    return t, s


def checksum(x: torch.Tensor) -> list[float]:
    """Order-independent fingerprints of a tensor (fp64 sum and sum of squares)."""
    d = x.detach().to(torch.float64)
    return [float(d.sum()), float((d * d).sum())]


def features(n: int, dim: int, seed: int, tokens: int = 729) -> tuple[torch.Tensor, torch.Tensor]:
    """Student / teacher post-LayerNorm outputs [n, tokens, dim] (for NT-Xent fixtures)."""
    g = torch.Generator().manual_seed(seed)
    s = _bf16(torch.randn(n, tokens, dim, generator=g))
    t = _bf16(torch.randn(n, tokens, dim, generator=g) + 0.5 * s)
    return s, t
