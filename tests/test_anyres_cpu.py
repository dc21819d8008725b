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
