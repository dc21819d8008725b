"""Host anyres pack plan vs transformers' pack_image_features (the code the reference calls)."""
import pytest
import torch

from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import anyres as A


@pytest.mark.parametrize("hw", [(336, 336), (480, 640), (640, 480), (300, 900), (1000, 500), (384, 384)])
def test_pack_map_matches_transformers(hw):
    from transformers import LlavaOnevisionConfig
    from transformers.models.llava_onevision.modeling_llava_onevision import (LlavaOnevisionModel,
                                                                              image_size_to_num_patches)
    cfg = LlavaOnevisionConfig()
    n = image_size_to_num_patches(list(hw), cfg.image_grid_pinpoints, 384)
    assert A.num_tiles(hw) == n
    m = LlavaOnevisionModel.__new__(LlavaOnevisionModel)
    m.config = cfg
    feats = [torch.arange(n * 729, dtype=torch.float64).view(n, 729, 1)]
    packed, lens = LlavaOnevisionModel.pack_image_features(m, feats, torch.tensor([hw]), image_newline=torch.full((1,), -1.0, dtype=torch.float64))
    ref = [int(v) for v in packed[0][:, 0].tolist()]
    mine = [-1 if e == -1 else e[0] * 729 + e[1] for e in A.pack_map(hw)]
    assert mine == ref


def test_kat9_token_counts():
    assert A.num_image_tokens((336, 336)) == 1485
    assert A.num_image_tokens((480, 640)) == 2929


def test_batch_maps_offsets():
    maps, lens = A.batch_maps([(336, 336), (336, 336)], tiles_per_sample=2)
    assert lens == [1485, 1485]
    assert maps[1][0] == 2 * 729 and maps[0][729] == 729 and maps[0][729 + 27] == -1


def test_library_pack_plan_matches_python():
    """kd_anyres_batch_map (C, for non-Python hosts) == anyres.batch_maps on a sweep of image
    sizes (aspect ratios from 1:6 to 6:1, odd sizes, the 336^2 bench size)."""
    import ctypes as C
    import numpy as np
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import _native as N
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import anyres
    sizes = [(336, 336), (480, 640), (640, 480), (300, 900), (1000, 500), (530, 730), (1, 1), (384, 2304),
             (2304, 384), (701, 233), (233, 701), (999, 1001), (1536, 1537), (17, 3000)]
    rng = np.random.default_rng(0)
    sizes += [(int(h), int(w)) for h, w in rng.integers(1, 2400, size=(200, 2))]
    for tiles in (37,):   # up to 6 x 6 + 1 tiles
        ok = []
        for hw in sizes:
            try:
                maps, lens = anyres.batch_maps([hw], tiles)
            except (NotImplementedError, ValueError):
                continue
            ok.append((hw, maps[0], lens[0]))
        B = len(ok)
        ld = max(l for _, _, l in ok)
        isz = np.array([hw for hw, _, _ in ok], dtype=np.int64)
        out = np.zeros((B, ld), dtype=np.int32)
        lens = np.zeros(B, dtype=np.int32)
        N.call("kd_anyres_batch_map", isz.ctypes.data, B, tiles, out.ctypes.data, ld, lens.ctypes.data)
        for b, (hw, m, n) in enumerate(ok):
            base = b * tiles * anyres.TOKENS_PER_TILE   # the C plan numbers rows over the whole batch
            ref = [(-1 if e == -1 else e + base) for e in m]
            assert lens[b] == n, hw
            assert out[b, :n].tolist() == ref, hw
            assert (out[b, n:] == -2).all()


def test_compact_tile_layout_c_equals_python():
    """tiles = 0: the feature rows of each sample follow the previous samples' REAL tiles (the
    vision tower runs only those, as HF's pix_val[:num_patch]); a mixed SUNRGBD-style batch
    [336x336 (2 tiles, 1485 tokens), 480x640 (5 tiles, 2929 tokens), 336x336]."""
    import numpy as np
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import _native as N
    sizes = [(336, 336), (480, 640), (336, 336)]
    maps, lens = A.batch_maps(sizes, 0)
    assert lens == [1485, 2929, 1485]
    assert maps[1][0] == 2 * 729 and maps[2][0] == (2 + 5) * 729
    assert max(v for v in maps[2] if v >= 0) < (2 + 5 + 2) * 729
    isz = np.array(sizes, dtype=np.int64)
    ld = max(lens)
    out = np.zeros((3, ld), dtype=np.int32)
    ln = np.zeros(3, dtype=np.int32)
    N.call("kd_anyres_batch_map", isz.ctypes.data, 3, 0, out.ctypes.data, ld, ln.ctypes.data)
    for b in range(3):
        assert ln[b] == lens[b] and out[b, :lens[b]].tolist() == maps[b] and (out[b, lens[b]:] == -2).all()
