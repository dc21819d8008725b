"""Drop-in KD LightningModules (the reference's L3 contract).

  OnlineKnowledgeDistillationLLavaOneVision   double-trouble module, phases 1/2/3 (DT)
  LogitBasedKD                                logit-based module, LoCa at T=1 (LB)
  FeatureBasedKD                              feature-based module (FB)
  LlavaOnevisionModule                        depth-student SFT baseline (BD)

Same constructor arguments, attributes (`student_model`, `teacher_model`, `phase`, `T`,
`gamma`, `soft_target_loss_weight`, `ce_loss_weight`, `learning_rate`), methods
(`training_step`, `validation_step`, `configure_optimizers`, `forward`, the freeze
helpers) and `self.log("train_loss" | "val_loss")` as the reference, and checkpoints
with `student_model.*` / `teacher_model.*` keys in the transformers-4.45 layout.

`training_step` returns a 0-d loss that requires grad; `loss.backward()` runs the
student backward (hand-written kernels, explicit order) into flat fp32 gradient
buffers, and the optimizer from `configure_optimizers()` is a fused AdamW over those
buffers.  Data-parallel ranks all-reduce the trainable gradient range in buckets as the
backward produces them (RCCL over xGMI).  Three streams per step: the teacher forward on
the main stream; the student forward, which does not read any teacher output, on a second
stream beside it (they fill each other's small-kernel gaps and GEMM wave-quantisation
tails); the AdamW and gradient zeroing of step t on a third, overlapping the teacher
forward of step t+1 (the student forward of step t+1 waits for them).
"""
from __future__ import annotations

import math
import os
import re

import torch
import torch.nn as nn

from . import ops
from .modeling import (STREAM_PRIORITY_HIGH, STUDENT_05B, TEACHER_7B, LlavaOnevisionModel, tiny_config)

try:  # the reference's base class when installed; otherwise a minimal stand-in
    import pytorch_lightning as _pl  # noqa: F401
    _Base = _pl.LightningModule
except Exception:  # pragma: no cover - pytorch_lightning is not in this image
    class _Base(nn.Module):
        def __init__(self):
            super().__init__()
            self.logged = {}

        def log(self, name, value, **kw):
            self.logged[name] = value


MODEL_CONFIGS = {
    "llava-hf/llava-onevision-qwen2-0.5b-ov-hf": STUDENT_05B,
    "llava-hf/llava-onevision-qwen2-7b-ov-hf": TEACHER_7B,
    "tiny-student": tiny_config(teacher=False),
    "tiny-teacher": tiny_config(teacher=True),
}


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("the KD step runs on the MI355X HIP kernels only (no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


class _KDStepFn(torch.autograd.Function):
    """Bridges Lightning's `loss.backward()` to the explicit student backward."""

    @staticmethod
    def forward(ctx, anchor, total, runner):
        ctx.runner = runner
        return total.clone()

    @staticmethod
    def backward(ctx, grad_out):
        ctx.runner._backward(grad_out.reshape(1).float().contiguous())
        ctx.runner = None
        return None, None, None


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics (DT:198-201) as one kernel over the trainable range."""

    def __init__(self, module, lr=1e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__([module._anchor], dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.module = module
        self.step_count = 0

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        m = self.module
        g = self.param_groups[0]
        self.step_count += 1
        m._finish_grad_sync()
        P = m.student_model.P
        lo, hi = m._trainable_range()
        if hi > lo:
            side = m._opt_stream
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                ops.adamw(P.master[lo:hi], P.flat[lo:hi], P.grad[lo:hi], P.exp_avg[lo:hi], P.exp_avg_sq[lo:hi],
                          g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"], self.step_count)
                m._opt_done.record(side)
            m._opt_pending = True
        return loss

    def zero_grad(self, set_to_none: bool = False):
        m = self.module
        lo, hi = m._trainable_range()
        if m._opt_pending:   # zero behind the AdamW on its stream; the next backward is ordered after it
            with torch.cuda.stream(m._opt_stream):
                m.student_model.P.grad[lo:hi].zero_()
                m._opt_done.record(m._opt_stream)
        else:
            m.student_model.P.grad[lo:hi].zero_()


class _KDBase(_Base):
    # subclass hooks
    uses_teacher = True

    def __init__(self, model_name_student, model_name_teacher, processor=None, learning_rate=1e-5, phase=1,
                 seed_teacher: int = 1, seed_student: int = 2, state_dict=None, world=None):
        super().__init__()
        self.phase = phase
        self.learning_rate = learning_rate
        self.processor = processor
        self.model_name_student, self.model_name_teacher = model_name_student, model_name_teacher
        dev = _device()
        small = model_name_student.startswith("tiny")
        self.student_model = LlavaOnevisionModel(MODEL_CONFIGS[model_name_student], dev, trainable=True,
                                                 seed=seed_student, cpu_rng=small)
        self.teacher_model = None
        if self.uses_teacher:
            self.teacher_model = LlavaOnevisionModel(MODEL_CONFIGS[model_name_teacher], dev, trainable=False,
                                                     seed=seed_teacher, cpu_rng=small)
        if state_dict is not None:
            self.load_kd_state_dict(state_dict)
        self.config = self.student_model.cfg
        self._anchor = nn.Parameter(torch.zeros((), device=dev))
        # the step's own streams run at high priority; the teacher prefetch (off the critical
        # path) at normal priority, so it fills the CUs the step leaves idle
        self._opt_stream = torch.cuda.Stream(device=dev, priority=STREAM_PRIORITY_HIGH)
        self._stu_stream = torch.cuda.Stream(device=dev, priority=STREAM_PRIORITY_HIGH)
        self.concurrent_student = True   # False: student forward on the main stream (bench.py --serial)
        self._opt_done = torch.cuda.Event()
        self._opt_pending = False
        self._tch_stream = torch.cuda.Stream(device=dev, priority=0)
        self.teacher_graphs = os.environ.get("KD_TEACHER_GRAPH", "0") == "1"   # measured slower on ROCm 7
        self._tgraphs = {}
        self._prefetched = None   # (batch key, teacher logits, post-LN features, event)
        self._ctx = None
        self.last_terms = None
        # data parallel
        import torch.distributed as dist
        self._dist = dist if (dist.is_available() and dist.is_initialized()) else None
        self._works = []
        self._sync_hi = None
        self._bucket_bytes = 256 << 20
        if self._dist is not None and self.uses_teacher:
            # teacher weights broadcast once from rank 0, then read-only in every GPU's HBM
            self._dist.broadcast(self.teacher_model.P.flat, src=0)
        if self._dist is not None:
            self._dist.broadcast(self.student_model.P.flat, src=0)
            self.student_model.P.master.copy_(self.student_model.P.flat.float())

    # ------------------------------------------------------------- freezing ----
    def _trainable_range(self):
        s = self.student_model
        R = s.P.regions
        parts = []
        if s.train_vision:
            parts.append(R["vision"])
        if s.train_projector:
            parts.append(R["projector"])
        if s.train_language:
            parts.append(R["language"])
        if not parts:
            return 0, 0
        lo, hi = min(p[0] for p in parts), max(p[1] for p in parts)
        if sum(p[1] - p[0] for p in parts) != hi - lo:
            raise RuntimeError("trainable regions must be contiguous (vision|projector|language)")
        return lo, hi

    def freeze_student_language_layers(self):            # DT:468-483
        self.student_model.train_language = False

    def unfreeze_student_language_layers(self):          # DT:486-499
        self.student_model.train_language = True

    def freeze_student_vision_layers(self):              # DT:501-508
        self.student_model.train_vision = False

    def unfreeze_student_vision_layers(self):            # DT:516-523
        self.student_model.train_vision = True

    def setup(self, stage=None):                         # DT:88-91
        pass

    # --------------------------------------------------------------- losses ----
    def _loss_spec(self):
        """(kd variant, T, kd_weight, ce_weight, ntxent weight or None)."""
        raise NotImplementedError

    def configure_optimizers(self):                      # DT:198-201
        opt = FusedAdamW(self, lr=self.learning_rate)
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
        return [opt], [sched]

    # ------------------------------------------------------------- the step ----
    @staticmethod
    def _batch_key(batch):
        # the input tensors themselves (held, so their memory cannot be reused by another
        # batch) and their version counters (an in-place edit invalidates the prefetch)
        x, p, sz = batch["rgb_input_ids"], batch["rgb_pixel_values"], batch["image_sizes"]
        return (x, p, sz, x._version, p._version)

    @staticmethod
    def _same_key(k1, k2):
        return all(a is b for a, b in zip(k1[:3], k2[:3])) and k1[3:] == k2[3:]

    def _teacher_forward_eager(self, batch, need_feats):
        tfwd = self.teacher_model.forward(batch["rgb_input_ids"], batch["rgb_pixel_values"], batch["image_sizes"],
                                          save=False, want_post_ln=need_feats)
        t_logits = self.teacher_model.logits(tfwd["hn"])
        del tfwd["hn"]
        return t_logits, tfwd.get("post_ln")

    def _teacher_forward(self, batch, need_feats):
        """Teacher logits (+ post-LN vision features) for `batch` on the current stream.

        The frozen teacher's forward is ~700 short host launches (~38 ms of Python + ctypes
        per step, which left the step close to launch-bound); it is captured once per input
        signature as a HIP graph (torch.cuda.CUDAGraph: every kernel is a libkdstep launch on
        the capturing stream) and replayed: one launch. The inputs are copied into the
        graph's static buffers; the outputs are the graph's static tensors (overwritten by
        the next replay, which every consumer precedes on the stream order)."""
        if not self.teacher_graphs:
            return self._teacher_forward_eager(batch, need_feats)
        ids, px, sz = batch["rgb_input_ids"], batch["rgb_pixel_values"], batch["image_sizes"]
        sizes = tuple(tuple(int(v) for v in hw) for hw in (sz.tolist() if hasattr(sz, "tolist") else sz))
        key = (tuple(ids.shape), tuple(px.shape), px.dtype, sizes, bool(need_feats))
        tg = self._tgraphs.get(key)
        if tg is None:
            out = self._teacher_forward_eager(batch, need_feats)   # warm-up: workspaces, maps, tables
            sb = dict(batch)
            sb["rgb_input_ids"], sb["rgb_pixel_values"] = ids.clone(), px.clone()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                logits, post = self._teacher_forward_eager(sb, need_feats)
            self._tgraphs[key] = (g, sb["rgb_input_ids"], sb["rgb_pixel_values"], logits, post)
            return out
        g, s_ids, s_px, logits, post = tg
        s_ids.copy_(ids)
        s_px.copy_(px)
        g.replay()
        return logits, post

    def prefetch_teacher(self, batch):
        """Enqueue the frozen teacher's forward for `batch` (the NEXT training batch) on its own
        stream, so it runs beside the current step's backward and optimizer; the
        training_step that gets this batch waits on it instead of recomputing it. Optional:
        without it the teacher runs inline. The teacher reads no student state, so the
        result is identical either way."""
        if not self.uses_teacher:
            return
        _, _, _, _, ctr_w = self._loss_spec()
        ts = self._tch_stream
        ts.wait_stream(torch.cuda.current_stream())   # the batch's inputs are ready
        with torch.cuda.stream(ts):
            t_logits, post_ln = self._teacher_forward(batch, ctr_w is not None)
        ev = torch.cuda.Event()
        ev.record(ts)
        self._prefetched = (self._batch_key(batch), t_logits, post_ln, ev)

    def _take_prefetched(self, batch, need_feats):
        pf, self._prefetched = self._prefetched, None
        if pf is None:
            return None
        _, t_logits, post_ln, ev = pf
        main = torch.cuda.current_stream()
        main.wait_event(ev)   # also when unused: an inline replay rewrites the same graph buffers
        if not self._same_key(pf[0], self._batch_key(batch)) or (need_feats and post_ln is None):
            return None
        # consumed on the main stream from here on: keep the allocator from handing the
        # blocks back to the teacher stream before those reads are done
        if not self.teacher_graphs:
            t_logits.record_stream(main)
            if post_ln is not None:
                post_ln.record_stream(main)
        return t_logits, post_ln

    def forward(self, batch, train: bool = False):
        """The reference's forward(batch) (DT:206-271): total loss as a 0-d fp32 tensor."""
        variant, T, kd_w, ce_w, ctr_w = self._loss_spec()
        labels = batch["labels"]
        image_sizes = batch["image_sizes"]
        B, L = batch["depth_input_ids"].shape
        need_feats = ctr_w is not None
        main = torch.cuda.current_stream()
        s = self.student_model
        # student forward on its own stream beside the teacher forward. It first waits for
        # everything already queued on the main stream (so caching-allocator blocks the
        # previous step freed there are reusable) and for the previous optimizer step (the
        # student weights); the main stream joins it before the loss. The teacher (the long
        # pole, ~90 ms of large GEMMs that do not read student weights) is ENQUEUED first:
        # the host spends ~20 ms launching the student's ~500 short kernels, and queued
        # first they ran alone on the GPU while the teacher's launches waited behind them.
        side = self._stu_stream if self.concurrent_student else main
        side.wait_stream(main)
        if self._opt_pending:
            side.wait_event(self._opt_done)
            self._opt_pending = False
        t_logits = t_post = None
        if self.uses_teacher:
            got = self._take_prefetched(batch, need_feats)
            t_logits, t_post = got if got is not None else self._teacher_forward(batch, need_feats)
        with torch.cuda.stream(side):
            sfwd = s.forward(batch["depth_input_ids"], batch["depth_pixel_values"], image_sizes, save=train,
                             want_post_ln=need_feats)
            s_logits = s.logits(sfwd["hn"])
        main.wait_stream(side)
        Vs = s_logits.shape[1]
        loss4, dlogits = ops.kd_loss_fwd_bwd(
            s_logits.view(B, L, Vs), None if t_logits is None else t_logits.view(B, L, -1), labels, variant,
            temperature=T, alpha=0.8, kd_weight=kd_w, ce_weight=ce_w, want_grad=train)
        del s_logits, t_logits
        total = loss4[3]
        dps = None
        if need_feats:
            NI = sfwd["post_ln"].shape[0] // s.cfg.vision.n_patches
            ps = ops.row_group_mean(sfwd["post_ln"], NI, s.cfg.vision.n_patches)        # DT:243-244
            pt = ops.row_group_mean(t_post, NI, s.cfg.vision.n_patches)
            ntx, dps = ops.ntxent(ps, pt, tau=0.07, weight=ctr_w, want_grad=train)      # DT:393-416
            total = total + ntx[0]
            self.last_ntxent = ntx
        self.last_terms = loss4
        if train:
            self._ctx = dict(sfwd=sfwd, dlogits=dlogits, dps=dps)
        return total

    def _backward(self, gscale):
        ctx, self._ctx = self._ctx, None
        s = self.student_model
        sf = ctx["sfwd"]
        hn = sf["hn"]
        W = s.lm_head_weight()
        dl = ctx["dlogits"].view(hn.shape[0], -1)
        dhn = ops.gemm(dl, W.t(), alpha_dev=gscale)                          # lm_head dgrad
        if s.train_language:                                                  # lm_head / tied embed wgrad
            ev = s.wlane.run(lambda: ops.gemm(dl.t(), hn.t(), out=s.lm_head_grad(), accumulate=True, alpha_dev=gscale),
                             dl, hn, gscale)
            if s.cfg.text.tie:
                s.tied_grad_event = ev
        del dl, ctx["dlogits"]
        dpost = None
        if ctx["dps"] is not None and s.train_vision:
            dpost = ops.row_group_mean_bwd(ctx["dps"], s.cfg.vision.n_patches, scale_dev=gscale)
        s.backward(sf, dhn, dpost, on_layer_done=self._on_layer_done if self._dist else None)
        self._launch_grad_sync(final=True)

    # ------------------------------------------------------- data parallel ----
    def _on_layer_done(self, i):
        """Bucketed all-reduce of LM grads as soon as the backward has made them final.

        Flat layout [vision | projector | embed, layers 0..N-1, norm(, lm_head)]; the backward
        finishes the tail first (lm_head, norm), then layers N-1..0, then embed / projector /
        vision.  Everything from layer i's first parameter to the current high-water mark is
        final once layer i is done."""
        s = self.student_model
        if not s.train_language:
            return
        P = s.P
        if self._sync_hi is None:
            self._sync_hi = P.numel
        first = P.offsets[f"language_model.model.layers.{i}.self_attn.q_proj.weight"][0]
        if (self._sync_hi - first) * 4 >= self._bucket_bytes:
            lane = getattr(s, "wlane", None)
            if lane is not None:
                lane.join()   # the bucket's weight grads (side stream) are complete
            self._allreduce(first, self._sync_hi)
            self._sync_hi = first

    def _launch_grad_sync(self, final: bool):
        if self._dist is None:
            return
        lo, hi = self._trainable_range()
        top = hi if self._sync_hi is None else min(hi, self._sync_hi)
        if top > lo:
            self._allreduce(lo, top)
        self._sync_hi = None

    def _allreduce(self, lo, hi):
        g = self.student_model.P.grad[lo:hi]
        if self._dist.get_backend() == "nccl":   # RCCL: AVG in the collective
            self._works.append((self._dist.all_reduce(g, op=self._dist.ReduceOp.AVG, async_op=True), None))
        else:                                      # gloo (CPU tests): SUM, divided after the wait
            self._works.append((self._dist.all_reduce(g, op=self._dist.ReduceOp.SUM, async_op=True), g))

    def _finish_grad_sync(self):
        ws = self._dist.get_world_size() if self._dist is not None else 1
        for w, g in self._works:
            w.wait()
            if g is not None:
                g.div_(ws)
        self._works = []

    # ---------------------------------------------------------- Lightning API ----
    def training_step(self, batch, batch_idx):           # DT:123-131
        total = self.forward(batch, train=True)
        loss = _KDStepFn.apply(self._anchor, total, self)
        self.log("train_loss", loss, on_step=True, on_epoch=True, prog_bar=True, logger=True)
        return loss

    def validation_step(self, batch, batch_idx):         # DT:133-138
        with torch.no_grad():
            loss = self.forward(batch, train=False)
        self.log("val_loss", loss, on_step=False, on_epoch=True, prog_bar=True, logger=True)
        return loss

    # ------------------------------------------------------------ checkpoints ----
    def kd_state_dict(self):
        if self._opt_pending:   # weights of a queued optimizer step
            torch.cuda.current_stream().wait_event(self._opt_done)
        sd = {f"student_model.{k}": v for k, v in self.student_model.P.state_dict().items()}
        if self.teacher_model is not None:
            sd.update({f"teacher_model.{k}": v for k, v in self.teacher_model.P.state_dict().items()})
        return sd

    def load_kd_state_dict(self, sd):
        self.student_model.P.load_state_dict(sd, prefix="student_model.")
        if self.teacher_model is not None and any(k.startswith("teacher_model.") for k in sd):
            self.teacher_model.P.load_state_dict(sd, prefix="teacher_model.")

    def save_checkpoint(self, path, epoch: int = 0, global_step: int = 0):
        """Lightning-style .ckpt: {'state_dict': {student_model.*, teacher_model.*}, ...}."""
        sd = {k: v.detach().cpu() for k, v in self.kd_state_dict().items()}
        torch.save({"state_dict": sd, "epoch": epoch, "global_step": global_step,
                    "pytorch-lightning_version": "2.4.0",
                    "hyper_parameters": {"model_name_student": self.model_name_student,
                                         "model_name_teacher": self.model_name_teacher,
                                         "learning_rate": self.learning_rate, "phase": self.phase}}, path)

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, model_name_student=None, model_name_teacher=None, processor=None,
                             map_location=None, **kw):
        ck = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        hp = ck.get("hyper_parameters", {})
        return cls(model_name_student or hp["model_name_student"], model_name_teacher or hp["model_name_teacher"],
                   processor, learning_rate=kw.pop("learning_rate", hp.get("learning_rate", 1e-5)),
                   state_dict=ck["state_dict"], **{k: v for k, v in kw.items() if k in ("phase",)})


class OnlineKnowledgeDistillationLLavaOneVision(_KDBase):
    """Double-trouble KD module (DT): phase 1 vision loss, 2 LoCa, 3 combined."""

    def __init__(self, model_name_student, model_name_teacher, processor=None, learning_rate=1e-5, phase=1, **kw):
        super().__init__(model_name_student, model_name_teacher, processor, learning_rate, phase, **kw)
        self.soft_target_loss_weight = 0.1   # DT:67-71
        self.ce_loss_weight = 0.5
        self.gamma = 0.8
        self.T = 0.8

    def _loss_spec(self):
        if self.phase == 1:   # compute_vision_loss: 0.1 KL T^2 + 0.5 NT-Xent, no CE (DT:316-354)
            return "kl", self.T, self.soft_target_loss_weight, 0.0, self.ce_loss_weight
        if self.phase == 2:   # compute_loca_loss + CE (DT:253-254)
            return "loca", self.T, 1.0, 1.0, None
        if self.phase == 3:   # gamma (loca + CE) + (1-gamma) CE (DT:257-260)
            return "loca", self.T, self.gamma, 1.0, None
        raise ValueError(f"phase {self.phase}")


class LogitBasedKD(_KDBase):
    """Logit-based module (LB): compute_loca_loss at T=1 (LB:164-165, :208-261)."""

    def __init__(self, model_name_student, model_name_teacher, processor=None, learning_rate=1e-5, **kw):
        super().__init__(model_name_student, model_name_teacher, processor, learning_rate, phase=0, **kw)
        self.soft_target_loss_weight = 0.5   # LB:73-75
        self.ce_loss_weight = 0.5
        self.T = 1.0

    def _loss_spec(self):
        return "loca", self.T, 1.0, 1.0, None


class FeatureBasedKD(_KDBase):
    """Feature-based module (FB): 0.1 KL(log_target quirk) T^2 + 0.8 CE + NT-Xent (FB:161-227)."""

    def __init__(self, model_name_student, model_name_teacher, processor=None, learning_rate=2e-5, **kw):
        super().__init__(model_name_student, model_name_teacher, processor, learning_rate, phase=0, **kw)
        self.soft_target_loss_weight = 0.1   # FB:72-74
        self.ce_loss_weight = 0.8
        self.T = 0.8

    def _loss_spec(self):
        return "kl_logtarget", self.T, self.soft_target_loss_weight, self.ce_loss_weight, 1.0

    def configure_optimizers(self):        # FB:233-234 (no scheduler)
        return FusedAdamW(self, lr=self.learning_rate)


class LlavaOnevisionModule(_KDBase):
    """Depth-student SFT baseline (BD:6-138): loss = the student's CE only."""
    uses_teacher = False

    def __init__(self, model_name, processor=None, learning_rate=2e-5, **kw):
        super().__init__(model_name, None, processor, learning_rate, phase=0, **kw)
        self.model = self.student_model

    def _loss_spec(self):
        return "none", 1.0, 0.0, 1.0, None

    def configure_optimizers(self):        # BD:137-138
        return FusedAdamW(self, lr=self.learning_rate)
