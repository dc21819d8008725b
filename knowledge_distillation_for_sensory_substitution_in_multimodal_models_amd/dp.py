"""Data-parallel gradient synchronisation of the student.

One process per GPU; the student's trainable gradient is one contiguous range of a flat
fp32 buffer (modeling.ParamStore), so the all-reduce (mean over ranks) is a handful of
large buckets, launched as soon as the backward has made a range final (LM layers
top-down, then embed_tokens / projector, then the SigLIP layers top-down: BackwardMarks),
overlapping the rest of the backward; RCCL over xGMI on GPUs (backend "nccl"),
gloo in the CPU tests.

Gradient accumulation (the reference trains with accumulate_grad_batches=64, DT1T:70,
:155): only the LAST micro-batch's backward of an optimizer step reduces, DDP `no_sync`
style — the earlier ones only accumulate locally.  No collective is ever in flight while
a backward writes the buffer: `begin()` retires pending work first.  With every
micro-batch's loss scaled by 1/k (Lightning), the reduced buffer is the mean over ranks of
the sum over micro-batches, i.e. the gradient of the global mean loss.

Volume (fp32 buckets, the default): the whole trainable range per optimizer step — 893.6 M
params = 3.57 GB at c4 (phase 3, LB, FB), 495.8 M = 1.98 GB at c3 (phase 2, ViT frozen); a
ring all-reduce moves 2 (N-1)/N of that per GPU (6.25 / 3.47 GB at N = 8).  comm_dtype =
torch.bfloat16 halves it: each bucket is cast to bf16 (kd_cast_f32_bf16) on the stream the
backward runs on, all-reduced in bf16, and cast back into the fp32 buffer (kd_cast_bf16_f32)
when the work is awaited; the summation then rounds to bf16 (~2^-9 relative per element).
fp32 stays the default: the reference accumulates its 64 micro-batches' gradients in fp32,
and the collective overlaps the backward and the next teacher forward either way.
"""
from __future__ import annotations

import re

# kd_model_backward's on_layer_done codes (include/kdstep.h, ABI 9): a Qwen2 layer index >= 0,
# or one of these for the parts the backward finishes after the language model
KD_CB_EMBED_PROJECTOR = -1


def KD_CB_VISION_LAYER(i: int) -> int:
    return -2 - i


class BackwardMarks:
    """Where the student gradient is final when kd_model_backward's callback fires.

    Flat layout [vision (embeddings, layers 0..V-1, post_layernorm) | projector, image_newline |
    language (embed_tokens, layers 0..N-1, norm)]; the backward finishes the language model top-down,
    then embed_tokens / projector, then the SigLIP layers top-down, the patch / position embeddings
    last.  first(code) is the flat offset from which everything up to the trainable range's top is
    final after callback `code` (offsets: ParamStore.offsets, name -> (offset, numel))."""

    def __init__(self, offsets: dict):
        self.lm, self.vis = {}, {}
        for name, (off, _) in offsets.items():
            mt = re.match(r"language_model\.model\.layers\.(\d+)\.", name)
            mv = re.match(r"vision_tower\.vision_model\.encoder\.layers\.(\d+)\.", name)
            if mt:
                i = int(mt.group(1))
                self.lm[i] = min(off, self.lm.get(i, off))
            elif mv:
                i = int(mv.group(1))
                self.vis[i] = min(off, self.vis.get(i, off))
        self.proj = min(off for name, (off, _) in offsets.items()
                        if name.startswith("multi_modal_projector.") or name == "image_newline")
        self.embed = offsets["language_model.model.embed_tokens.weight"][0]

    def first(self, code: int, train_language: bool, train_projector: bool, train_vision: bool):
        """The flat offset, or None when `code` finishes nothing trainable."""
        if code >= 0:
            return self.lm[code] if train_language else None
        if code == KD_CB_EMBED_PROJECTOR:
            if train_projector:
                return self.proj
            return self.embed if train_language else None
        i = -2 - code
        return self.vis[i] if train_vision else None


class GradSync:
    """Bucketed all-reduce of `grad` (a flat tensor) over the default process group.

    Protocol per backward:   begin(sync) -> layer_done(first)* -> end(lo, hi)
    before the optimizer:    finish(lo, hi)
    """

    def __init__(self, dist, grad, bucket_bytes: int = 256 << 20, comm_dtype=None):
        self.dist = dist
        self.grad = grad
        self.bucket_bytes = int(bucket_bytes)
        self.comm_dtype = comm_dtype   # None: reduce the fp32 buffer in place; torch.bfloat16: bf16 buckets
        self.works = []          # (work, fp32 range view, bf16 comm buffer | None)
        self.hi = None           # high-water mark: [first, hi) already launched this backward
        self.active = False      # this backward reduces
        self.unsynced = False    # local grads accumulated since the last reduction
        self.world = dist.get_world_size()
        self.avg_in_collective = dist.get_backend() == "nccl"   # RCCL AVG; gloo has no AVG
        self.last_buckets = []   # element counts of the buckets of the last reducing backward
        self.last_tail = 0       # elements of those launched only by end(), after the backward
        self._cur_buckets = []
        self.top = None          # the trainable range's top (begin): nothing above it is reduced

    # -------------------------------------------------------------- backward ----
    def begin(self, sync: bool, top: int | None = None):
        self.wait()              # nothing in flight while this backward accumulates into grad
        self.active = bool(sync)
        self.hi = None
        self.top = top
        self._cur_buckets = []

    def layer_done(self, first: int, before_launch=None):
        """Everything from flat offset `first` to the high-water mark is final."""
        if not self.active:
            return
        if self.hi is None:
            self.hi = self.grad.numel() if self.top is None else self.top
        if first >= self.hi:
            return
        if (self.hi - first) * self.grad.element_size() >= self.bucket_bytes:
            if before_launch is not None:
                before_launch()  # e.g. join the weight-gradient stream
            self._launch(first, self.hi)
            self.hi = first

    def end(self, lo: int, hi: int):
        """The backward is complete: reduce what is left of the trainable range [lo, hi)."""
        if self.active:
            top = hi if self.hi is None else min(hi, self.hi)
            self.last_tail = max(0, top - lo)
            if top > lo:
                self._launch(lo, top)
            self.unsynced = False
            self.last_buckets = list(self._cur_buckets)
        else:
            self.unsynced = True
        self.active = False
        self.hi = None

    # ------------------------------------------------------------- optimizer ----
    def finish(self, lo: int, hi: int):
        """Before the optimizer reads grad: reduce grads accumulated without a sync (an
        optimizer step taken before the accumulation boundary) and retire all work."""
        if self.unsynced and hi > lo:
            self._launch(lo, hi)
        self.unsynced = False
        self.wait()

    def wait(self):
        for w, g, buf in self.works:
            w.wait()
            if buf is not None:   # bf16 bucket back into the fp32 buffer
                if g.is_cuda:
                    import torch
                    from . import ops
                    ops.cast_bf16_f32(buf, g)
                    # the bucket was allocated on the backward's stream; this cast runs on the
                    # awaiting one (the optimizer's): keep the block until the cast has read it
                    buf.record_stream(torch.cuda.current_stream())
                else:
                    g.copy_(buf)
            if not self.avg_in_collective:
                g.div_(self.world)   # gloo: SUM, divided once (each range is reduced once per sync)
        self.works = []

    def _launch(self, lo: int, hi: int):
        g = self.grad[lo:hi]
        d = self.dist
        buf = None
        if self.comm_dtype is not None:
            import torch
            buf = torch.empty(g.numel(), dtype=self.comm_dtype, device=g.device)
            if g.is_cuda:
                from . import ops
                ops.cast_f32_bf16(g, buf)
            else:
                buf.copy_(g)
        t = g if buf is None else buf
        self._cur_buckets.append(int(g.numel()))
        op = d.ReduceOp.AVG if self.avg_in_collective else d.ReduceOp.SUM
        self.works.append((d.all_reduce(t, op=op, async_op=True), g, buf))
