"""Host-side logic of the drop-in module that needs no GPU: the transformers key layouts
 and the refusal of the reference's fp16 GradScaler mode (DT1T:147)."""
import pytest
import torch

from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd import kd_module as K
from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (
    ParamStore, hf_state_dict_to_445, hub_key_to_445, tiny_config)


def _hf5_model(cfg):
    from transformers import LlavaOnevisionConfig, LlavaOnevisionForConditionalGeneration
    V, T = cfg.vision, cfg.text
    hc = LlavaOnevisionConfig(
        vision_config=dict(model_type="siglip_vision_model", hidden_size=V.hidden, intermediate_size=V.inter,
                           num_hidden_layers=V.layers, num_attention_heads=V.heads, patch_size=V.patch,
                           image_size=V.image, vision_use_head=False, layer_norm_eps=V.eps),
        text_config=dict(model_type="qwen2", hidden_size=T.hidden, intermediate_size=T.inter,
                         num_hidden_layers=T.layers, num_attention_heads=T.heads, num_key_value_heads=T.kv_heads,
                         vocab_size=T.vocab, tie_word_embeddings=T.tie, rope_theta=T.rope_theta,
                         rms_norm_eps=T.eps, max_position_embeddings=4096),
        tie_word_embeddings=T.tie)
    return LlavaOnevisionForConditionalGeneration(hc)


@pytest.mark.parametrize("teacher", [False, True])
def test_installed_transformers_state_dict_loads_by_4_45_names(teacher):
    """A transformers-5.x state_dict (installed layout) renamed by the package's map fills
    every parameter of the 4.45 layout, value for value."""
    cfg = tiny_config(teacher)
    hf = _hf5_model(cfg)
    sd = {k: v.detach() for k, v in hf.state_dict().items()}
    P = ParamStore(cfg, "cpu")
    seen = P.load_state_dict(hf_state_dict_to_445(sd), strict=True)
    assert len(seen) == len(P.specs)
    w = P["language_model.model.layers.1.mlp.down_proj.weight"].float()
    ref = sd["model.language_model.layers.1.mlp.down_proj.weight"].bfloat16().float()
    assert torch.equal(w, ref)
    q = P["vision_tower.vision_model.encoder.layers.0.self_attn.q_proj.weight"].float()
    assert torch.equal(q, sd["model.vision_tower.encoder.layers.0.self_attn.q_proj.weight"].bfloat16().float())


def test_key_map_both_layouts():
    four45 = ["vision_tower.vision_model.post_layernorm.weight", "multi_modal_projector.linear_1.bias",
              "image_newline", "language_model.model.norm.weight", "language_model.lm_head.weight"]
    five = ["model.vision_tower.post_layernorm.weight", "model.multi_modal_projector.linear_1.bias",
            "model.image_newline", "model.language_model.norm.weight", "lm_head.weight"]
    for a, b in zip(four45, five):
        assert hub_key_to_445(a) == a       # the reference's (and the hub's) layout passes through
        assert hub_key_to_445(b) == a
    with pytest.raises(KeyError):
        hf_state_dict_to_445({"lm_head.weight": 0, "language_model.lm_head.weight": 1})


@pytest.mark.parametrize("p", ["16", "16-mixed", "16-true"])
def test_fp16_trainer_precision_is_refused(p):
    with pytest.raises(ValueError, match="bf16-true"):
        K.check_trainer_precision(p)


@pytest.mark.parametrize("p", [None, "bf16-true", "bf16-mixed", "32-true", "32", 32])
def test_bf16_and_fp32_precisions_accepted(p):
    K.check_trainer_precision(p)


def test_grad_scaler_step_is_refused():
    class _M:
        _anchor = torch.nn.Parameter(torch.zeros(()))
    opt = K.FusedAdamW(_M())
    scaler = torch.amp.GradScaler("cpu")
    loss = (_M._anchor * 2).sum()
    scaler.scale(loss).backward()
    with pytest.raises(RuntimeError, match="GradScaler"):
        scaler.step(opt)
