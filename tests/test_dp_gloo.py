"""Data-parallel gradient sync (dp.GradSync), world_size 2 on the gloo backend (CPU).

Each rank runs k micro-batch "backwards" that accumulate into a flat fp32 gradient
buffer the way the student backward does (top-down layer callbacks, then the rest),
with only the last one reducing (accumulate_grad_batches / no_sync semantics, DT1T:155).
After finish(), every rank must hold the mean over ranks of its local sum — each range
reduced exactly once, frozen ranges untouched."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _layout(train_vision, train_language):
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.modeling import (param_specs,
                                                                                                   tiny_config)
    cfg = tiny_config(False)
    offsets, off = {}, 0
    for s in param_specs(cfg):
        n = int(np.prod(s.shape))
        off = (off + 7) // 8 * 8
        offsets[s.name] = (off, n)
        off += n
    numel = (off + 7) // 8 * 8
    first_proj = offsets["multi_modal_projector.linear_1.weight"][0]
    first_lm = offsets["language_model.model.embed_tokens.weight"][0]
    parts = []
    if train_vision:
        parts.append((0, first_proj))
    parts.append((first_proj, first_lm))
    if train_language:
        parts.append((first_lm, numel))
    lo, hi = min(p[0] for p in parts), max(p[1] for p in parts)
    return cfg, offsets, numel, lo, hi


def _worker(rank, world, port, q, train_vision, train_language, k_micro, early_step, comm_bf16=False):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd.dp import (
        KD_CB_EMBED_PROJECTOR, KD_CB_VISION_LAYER, BackwardMarks, GradSync)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, offsets, numel, lo, hi = _layout(train_vision, train_language)
    grad = torch.zeros(numel)
    gs = GradSync(dist, grad, bucket_bytes=64 << 10, comm_dtype=torch.bfloat16 if comm_bf16 else None)
    g = torch.Generator().manual_seed(100 + rank)
    local = torch.zeros(numel)
    n_back = k_micro - 1 if early_step else k_micro
    marks = BackwardMarks(offsets)
    # kd_model_backward's callback order (include/kdstep.h ABI 9): Qwen2 layers top-down, then
    # embed_tokens / projector, then the SigLIP layers top-down; the patch embeddings last
    codes = list(reversed(range(cfg.text.layers))) + [KD_CB_EMBED_PROJECTOR] + \
        [KD_CB_VISION_LAYER(i) for i in reversed(range(cfg.vision.layers))]
    in_backward = 0
    for mb in range(n_back):
        sync = (mb == k_micro - 1)
        gs.begin(sync, top=hi)
        contrib = torch.randn(numel, generator=g) / k_micro       # loss / accumulate_grad_batches
        contrib[:lo] = 0
        contrib[hi:] = 0
        local += contrib
        # the backward writes top-down; a reduced range must already hold its final value
        top = offsets["language_model.model.norm.weight"][0]
        grad[top:] += contrib[top:]
        for code in codes:
            part = marks.first(code, True, True, True)      # where this part's gradient starts
            grad[part:top] += contrib[part:top]
            top = part
            first = marks.first(code, train_language, True, train_vision)
            if first is not None:
                gs.layer_done(first)
        grad[:top] += contrib[:top]
        in_backward = len(gs.works)
        gs.end(lo, hi)
        if not sync:
            assert not gs.works, "a non-final micro-batch must not launch a collective"
    tail = gs.last_tail
    gs.finish(lo, hi)
    q.put((rank, local.numpy(), grad.numpy().copy(), (lo, hi), (tail, in_backward, marks.vis[0], gs.bucket_bytes)))
    dist.destroy_process_group()


@pytest.mark.parametrize("train_vision,train_language,k_micro,early_step,comm_bf16",
                         [(True, True, 1, False, False), (False, True, 3, False, False), (True, False, 2, False, False),
                          (True, True, 3, True, False), (True, True, 2, False, True)])
def test_accumulated_grads_reduced_once_at_the_boundary(train_vision, train_language, k_micro, early_step, comm_bf16):
    """comm_bf16: bf16 buckets (GradSync comm_dtype): the mean within bf16 rounding."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (hash((train_vision, train_language, k_micro, early_step, comm_bf16)) % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, train_vision, train_language, k_micro, early_step,
                                               comm_bf16))
             for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (torch.from_numpy(b), torch.from_numpy(a), rng, bk)) for r, b, a, rng, bk in
               (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lo, hi = res[0][2]
    mean = (res[0][0] + res[1][0]) / 2
    # the buckets are launched as the backward makes them final: what end() launches after the
    # backward is less than one bucket above the SigLIP patch / position embeddings (the ViT, the
    # projector and embed_tokens no longer wait for the whole backward)
    tail, in_backward, vis_embed_elems, bucket_bytes = res[0][3]
    if not early_step:   # (an early optimizer step reduces in finish(), after no reducing backward)
        assert tail * 4 < bucket_bytes + 4 * (vis_embed_elems if train_vision else 0), (tail, bucket_bytes)
        assert in_backward >= 1
    for r in (0, 1):
        local, after, _, _ = res[r]
        if comm_bf16:   # each rank's sum rounded to bf16, then the bf16 sum: ~3 half-ulps of the result
            err = (after[lo:hi] - mean[lo:hi]).abs()
            scale = res[0][0][lo:hi].abs() + res[1][0][lo:hi].abs()
            assert bool((err <= 2.0 ** -8 * scale + 1e-30).all()), float((err / (scale + 1e-30)).max())
            assert torch.equal(res[0][1][lo:hi], res[1][1][lo:hi])   # replicas agree exactly
        else:
            assert torch.allclose(after[lo:hi], mean[lo:hi], atol=1e-6)
        assert float(after[:lo].abs().sum()) == 0.0 and float(after[hi:].abs().sum()) == 0.0
