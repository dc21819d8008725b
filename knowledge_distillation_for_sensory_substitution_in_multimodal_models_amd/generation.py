"""Student generate(): prefill + KV-cache greedy decode on the HIP kernels.

Drop-in for the call the reference's evaluation makes on the trained student
(evaluation/onevisionv3/evaluate_onevision.py:185-195):

    model.generate(**inputs, max_new_tokens=32, pad_token_id=pad_token_id,
                   repetition_penalty=1.2, no_repeat_ngram_size=2, temperature=0.7)

`do_sample` is not set there, so decoding is greedy and `temperature` has no effect (transformers
only applies it when sampling).  The prompt runs through the same forward as training
(LlavaOnevisionModel.forward: SigLIP, projector, anyres pack, Qwen2), whose roped keys and values
seed a per-layer KV cache [HKV, L + max_new_tokens, hd]; each new token then runs one row through
every layer (kd_gemv with the RMSNorms fused in front and bias / residual / SwiGLU epilogues, kd_qkv_split with its
RoPE row, split-KV kd_attn_decode) and kd_gen_select picks it on the device.  The position lives in a device counter, so
every launch of a step has fixed arguments: the first step runs eagerly, the step is captured
once as a HIP graph (torch.cuda.CUDAGraph) and replayed for the rest; steps past an EOS are
discarded afterwards (one host read at the end instead of one per token).  Returns prompt + generated ids like
transformers' generate (B = 1, as the evaluation runs it).
"""
from __future__ import annotations

import torch

from . import ops


EOS_TOKEN_IDS = (151645,)   # <|im_end|>: generation_config.eos_token_id of the -ov-hf chat checkpoints


FUSE_NORM_DEFAULT = True   # RMSNorm fused into the decode GEMVs (tools/bench_generate.py passes fuse_norm for A/B)


@torch.no_grad()
def generate(model, input_ids: torch.Tensor, pixel_values: torch.Tensor, image_sizes, max_new_tokens: int = 32,
             repetition_penalty: float = 1.0, no_repeat_ngram_size: int = 0, eos_token_id=EOS_TOKEN_IDS,
             pad_token_id: int | None = None, temperature: float | None = None, return_logits: bool = False,
             graph: bool = True, fuse_norm: bool | None = None):
    """-> int64 [1, L + n_new] on the device (and the bf16 logits row of every step if
    return_logits).  `temperature` is accepted for signature parity and ignored (greedy).
    fuse_norm: RMSNorm fused into the q|k|v and gate|up GEMVs (default: FUSE_NORM_DEFAULT)."""
    del temperature, pad_token_id   # greedy, batch of one: no padding of finished rows
    FUSE_NORM = FUSE_NORM_DEFAULT if fuse_norm is None else bool(fuse_norm)
    if input_ids.dim() != 2 or input_ids.shape[0] != 1:
        raise ValueError("generate: batch size 1 (as evaluate_onevision.py runs it)")
    T, P = model.cfg.text, model.P
    dev = model.device
    L = int(input_ids.shape[1])
    smax = L + int(max_new_tokens)
    eos = {int(e) for e in ([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or ()))}
    nq, nkv, hd = T.heads, T.kv_heads, T.head_dim
    qd, kd = nq * hd, nkv * hd
    lp = "language_model.model."

    # ---- prefill: the training forward, its roped k/v kept
    kv = []
    fwd = model.forward(input_ids, pixel_values, image_sizes, save=False, kv_out=kv)
    kc = torch.empty((T.layers, nkv, smax, hd), dtype=torch.bfloat16, device=dev)
    vc = torch.empty_like(kc)
    for i, (k, v) in enumerate(kv):
        kc[i, :, :L].copy_(k[0])
        vc[i, :, :L].copy_(v[0])
    del kv
    seq = torch.empty(smax, dtype=torch.int64, device=dev)
    seq[:L].copy_(input_ids[0])
    logits = model.logits(fwd["hn"][L - 1:L])
    del fwd
    steps = [logits] if return_logits else None
    ops.gen_select(logits, seq, L, repetition_penalty, no_repeat_ngram_size)

    cos, sin = model._rope_for(smax)
    src = torch.full((1,), -2, dtype=torch.int32, device=dev)   # token embedding (kd_embed_assemble)
    table = P[lp + "embed_tokens.weight"]
    layers = []
    for i in range(T.layers):
        p = f"{lp}layers.{i}."
        layers.append((P[p + "input_layernorm.weight"],
                       P.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight", qd + 2 * kd, T.hidden),
                       P.span(p + "self_attn.q_proj.bias", p + "self_attn.v_proj.bias", 1, qd + 2 * kd).view(-1),
                       P[p + "self_attn.o_proj.weight"], P[p + "post_attention_layernorm.weight"],
                       P.span(p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight", 2 * T.inter, T.hidden),
                       P[p + "mlp.down_proj.weight"]))
    # device-resident step state: the sequence length (tokens so far, the one being decoded
    # included), the token being decoded and its RoPE row -> every launch of a step has fixed
    # arguments and the step replays from one captured HIP graph
    cur = torch.full((1,), L + 1, dtype=torch.int32, device=dev)
    tok = seq[L:L + 1].clone()   # the token being decoded (kd_gen_select rewrites it each step)
    cos_row = torch.empty((1, cos.shape[1]), dtype=torch.float32, device=dev)
    sin_row = torch.empty_like(cos_row)

    def step():
        ops.rope_row(cos, sin, cur, cos_row, sin_row)
        x = ops.embed_assemble(tok, src, table, None, None, model.err)
        for i, (w_in, Wqkv, bqkv, Wo, w_post, Wgu, Wdown) in enumerate(layers):
            if FUSE_NORM:
                qkv = ops.gemv(x, Wqkv, bias=bqkv, norm_w=w_in, eps=T.eps)      # input_layernorm fused
            else:
                h, _, _ = ops.norm_fwd(x, w_in, None, T.eps, rms=True, save_stats=False)
                qkv = ops.gemv(h, Wqkv, bias=bqkv)
            q, k, v = ops.qkv_split(qkv, 1, 1, nq, nkv, hd, hd, cos_row, sin_row)
            o = ops.attn_decode(q.view(nq, hd), k.view(nkv, hd), v.view(nkv, hd), kc[i], vc[i], 0, hd, cur=cur)
            x_mid = ops.gemv(o, Wo, residual=x)
            if FUSE_NORM:
                a = ops.gemv(x_mid, Wgu, swiglu_inter=T.inter, norm_w=w_post, eps=T.eps)  # post_attention_layernorm
            else:
                h2, _, _ = ops.norm_fwd(x_mid, w_post, None, T.eps, rms=True, save_stats=False)
                a = ops.gemv(h2, Wgu, swiglu_inter=T.inter)
            x = ops.gemv(a, Wdown, residual=x_mid)
        # final norm as its own launch: fused into the 38k-workgroup lm_head GEMV it would be recomputed
        # by every workgroup (measured slower)
        hn, _, _ = ops.norm_fwd(x, P[lp + "norm.weight"], None, T.eps, rms=True, save_stats=False)
        lg = ops.gemv(hn, model.lm_head_weight())
        ops.gen_select(lg, seq, 0, repetition_penalty, no_repeat_ngram_size, out=tok, cur=cur)
        return lg

    n_steps = smax - (L + 1)
    graph_obj = None
    for t_ in range(n_steps):
        if graph and t_ == 1:   # step 0 ran eagerly (warm-up: allocations, workspaces); capture the rest
            graph_obj = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph_obj):
                lg_static = step()
        if graph_obj is not None:
            graph_obj.replay()
            lg = lg_static
        else:
            lg = step()
        if return_logits:
            steps.append(lg.clone())
    n = smax
    if eos:   # transformers stops after the first EOS; the steps past it are discarded
        gen = seq[L:smax].tolist()
        for j, t_ in enumerate(gen):
            if t_ in eos:
                n = L + j + 1
                break
        if return_logits:
            steps = steps[:n - L]
    out = seq[:n].view(1, n)
    return (out, steps) if return_logits else out
