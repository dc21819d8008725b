"""ORACLE — test infrastructure only, never the product path.

CPU restatement of the token choice transformers' generate() makes for the reference's
evaluation call (evaluation/onevisionv3/evaluate_onevision.py:185-195: greedy, repetition_penalty
=1.2, no_repeat_ngram_size=2): RepetitionPenaltyLogitsProcessor, NoRepeatNGramLogitsProcessor,
then argmax of the float32 scores.  Checked against transformers' own processor classes
(tests/test_generate.py).  Only tests/ may import this module.
"""
from __future__ import annotations

import numpy as np


def process_scores(scores: np.ndarray, seq, penalty: float, ngram: int) -> np.ndarray:
    """scores [V] float32, seq = all ids so far (prompt + generated) -> processed float32 scores."""
    s = scores.astype(np.float32).copy()
    seq = [int(t) for t in seq]
    if penalty != 1.0:
        ids = np.unique(np.array(seq, dtype=np.int64))
        g = s[ids]
        s[ids] = np.where(g < 0, g * np.float32(penalty), g / np.float32(penalty)).astype(np.float32)
    n = len(seq)
    if ngram > 0 and n + 1 >= ngram:
        prefix = tuple(seq[n - ngram + 1:])
        for i in range(0, n - ngram + 1):
            if tuple(seq[i:i + ngram - 1]) == prefix:
                s[seq[i + ngram - 1]] = -np.inf
    return s


def select(scores: np.ndarray, seq, penalty: float, ngram: int) -> int:
    return int(np.argmax(process_scores(scores, seq, penalty, ngram)))
