"""Loader for the committed KD-loss fixtures (tests/golden/kd_*.npz)."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import torch

import inputs as I

HERE = Path(__file__).resolve().parent


def kd_fixture_names():
    return sorted(p.stem[3:] for p in HERE.glob("kd_*.npz"))


def load_kd_fixture(name):
    z = np.load(HERE / f"kd_{name}.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return meta, {k: z[k] for k in z.files if k != "meta"}


def make_labels(rec):
    """Same recipe as make_golden.make_labels (kept here so the box needs no reference)."""
    B, L, seed = rec["B"], rec["L"], rec["seed"]
    if rec["labels"] == "layout":
        return I.token_ids(B, L, seed=seed, n_image=min(I.N_IMAGE_TOKENS_336, L - 40))
    if rec["labels"] == "random":
        g = torch.Generator().manual_seed(seed + 1000)
        return torch.randint(0, 64, (B, L), generator=g) * 2371
    if rec["labels"] == "pad":
        ids = I.token_ids(B, L, seed=seed, n_image=min(I.N_IMAGE_TOKENS_336, L - 40))
        ids[1, L - 100:] = -100
        return ids
    raise ValueError(rec["labels"])


def kd_inputs(meta, exp=None):
    labels = make_labels(meta)
    t, s = I.kd_logits(meta["B"], meta["L"], meta["seed"], labels.clamp(min=0))
    if exp is not None:
        for key, x in (("t_ck", t), ("s_ck", s), ("labels_ck", labels)):
            got = np.array(I.checksum(x))
            assert np.allclose(got, exp[key], rtol=1e-12, atol=0), f"input regeneration drifted: {key}"
    return t, s, labels


VARIANT_OF = {"loca": "loca", "kl": "kl", "kllt": "kl_logtarget", "ce": "none"}
