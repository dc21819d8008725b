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

import contextlib
import inspect


import torch
import torch.nn as nn

from . import ops
from .dp import BackwardMarks, GradSync
from .modeling import (STREAM_PRIORITY_HIGH, STUDENT_05B, TEACHER_7B, LlavaOnevisionModel, real_width_config,
                       tiny_config)

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
    # the real widths at 2 layers per tower (model-level parity fixtures, tests/golden/model_real_*)
    "real2-student": real_width_config(teacher=False, layers=2),
    "real2-teacher": real_width_config(teacher=True, layers=2),
}
# the public checkpoints' names: weights too large for the CPU RNG (device RNG instead)
_HUB_NAMES = ("llava-hf/llava-onevision-qwen2-0.5b-ov-hf", "llava-hf/llava-onevision-qwen2-7b-ov-hf")


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


_FP16_MSG = ("the MI355X KD step trains in bf16 with fp32 master weights (no loss scaling); the reference's "
             "fp16 autocast + GradScaler mode (Trainer precision=\"16\", DT1T:147) is not supported: use "
             "precision=\"bf16-true\" (INTEGRATION.md)")


def check_trainer_precision(precision) -> None:
    """Reject the fp16 modes (precision "16", "16-mixed", "16-true"): a GradScaler would scale
    the loss and then look for torch .grad tensors the fused optimizer never creates."""
    p = str(precision if precision is not None else "").strip().lower()
    if p == "16" or p.startswith("16-") or p in ("fp16", "half"):
        raise ValueError(_FP16_MSG)


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics (DT:198-201) as one kernel over the trainable range."""

    # GradScaler.step hands itself to a step() that takes `grad_scaler`: the fp16 path is
    # then refused here with a clear error instead of an assertion inside the scaler
    _step_supports_amp_scaling = True

    def __init__(self, module, lr=1e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__([module._anchor], dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.module = module
        self.step_count = 0

    @torch.no_grad()
    def step(self, closure=None, grad_scaler=None):
        # GradScaler passes itself (torch 2.x), or sets grad_scale / found_inf (announced)
        if grad_scaler is not None or getattr(self, "grad_scale", None) is not None:
            raise RuntimeError(_FP16_MSG)
        loss = closure() if closure is not None else None
        m = self.module
        g = self.param_groups[0]
        # a batch the reference would have rejected (label out of range, DT:166) never
        # updates the weights: the kernel skips on the step's sticky error words (device
        # side, no host wait); the host raises as soon as it sees them
        m._check_errors(block=False)
        lo, hi = m._trainable_range()
        # the student stream (beside the next teacher forward); the caller's stream when
        # the module runs serialized (bench.py --serial, measurement)
        side = m._opt_stream if m.concurrent_student else torch.cuda.current_stream()
        side.wait_stream(torch.cuda.current_stream())
        if m._bwd_pending:   # the backward runs on its own stream
            side.wait_event(m._bwd_done)
        if m._gsync is not None:
            # the all-reduce's completion is awaited on the student stream only: the caller's
            # stream (the next teacher forward) does not queue behind the collective
            with torch.cuda.stream(side):
                m._gsync.finish(lo, hi)
        m._micro = 0
        self.step_count += 1
        P = m.student_model.P
        if hi > lo:
            with torch.cuda.stream(side):
                # the error words as of this step's loss (a snapshot taken on the main stream
                # right after it): the live words may already carry the NEXT step's teacher
                # error (its forward runs on the main stream beside this AdamW), which must not
                # cancel this valid step's update
                skip = m._errors.snapshot if m._errors.snapshot is not None else m._errors.words
                ops.adamw(P.master[lo:hi], P.flat[lo:hi], P._grad[lo:hi], P.exp_avg[lo:hi], P.exp_avg_sq[lo:hi],
                          g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"], self.step_count,
                          skip_words=skip)
                skip.record_stream(side)   # allocated on the main stream
                m._opt_done.record(side)
            m._opt_pending = True
        return loss

    def zero_grad(self, set_to_none: bool = False):
        m = self.module
        lo, hi = m._trainable_range()
        if m._opt_pending and m.concurrent_student:   # zero behind the AdamW on its stream
            with torch.cuda.stream(m._opt_stream):
                ops.zero_(m.student_model.P._grad[lo:hi])
                m._opt_done.record(m._opt_stream)
        else:
            ops.zero_(m.student_model.P.grad[lo:hi])


class _ErrorWatch:
    """Device error words of a step (label range in the KD loss, token ids / image-token
    count in the embedding assembly) in one int32 buffer: [0:4] kd_loss_params.err_out,
    [4] the student's embedding error, [5] the teacher's.  The words are STICKY (never
    reset on the device until the host has reported them) and kd_adamw reads them as its
    skip words, so a batch the reference would have rejected (DT:166) leaves the weights
    untouched, and so does every step queued behind it — the state the reference's
    RuntimeError leaves.  The host side is asynchronous: after each step's loss the words
    are copied into a pinned slot and an event is recorded; training_step / optimizer.step
    raise for any completed slot (no wait), validation_step and check(block=True) wait."""

    SLOTS = 4

    def __init__(self, dev):
        self.words = torch.zeros(8, dtype=torch.int32, device=dev)
        self.kd = self.words[0:4]
        self.snapshot = None  # the words as of the last step's loss (kd_adamw's skip words)
        self.host = torch.zeros((self.SLOTS, 6), dtype=torch.int32).pin_memory()
        self.pending = []    # (event, slot, info)
        self.next = 0

    def bind(self, student, teacher):
        """Point the models' embedding error words into the buffer."""
        student.err = self.words[4:5]
        if teacher is not None:
            teacher.err = self.words[5:6]

    def record(self, info):
        """Enqueue the copy on the current stream (after the step's loss)."""
        if len(self.pending) >= self.SLOTS:
            self.check(block=True, upto=1)
        slot = self.next
        self.next = (self.next + 1) % self.SLOTS
        # device snapshot for this step's AdamW (ordered after this step's loss and teacher
        # forward, before the next step's teacher forward: all on this stream)
        self.snapshot = self.words.clone()
        self.host[slot].copy_(self.words[0:6], non_blocking=True)
        ev = torch.cuda.Event(blocking=True)   # a host wait on it sleeps instead of spinning
        ev.record()
        self.pending.append((ev, slot, info))

    def check(self, block: bool, upto: int | None = None):
        keep = []
        for i, (ev, slot, info) in enumerate(self.pending):
            if (block and (upto is None or i < upto)) or ev.query():
                ev.synchronize()
                h = self.host[slot].tolist()
                if any(h):
                    # reported once: later slots hold the same sticky words
                    self.pending = []
                    torch.cuda.synchronize()
                    self.words.zero_()
                    if self.snapshot is not None:
                        self.snapshot.zero_()
                    self._raise_if(h, info)
            else:
                keep.append((ev, slot, info))
        self.pending = keep

    @staticmethod
    def _raise_if(h, info):
        bits, lab, row, _, serr, terr = h
        L, V = info["L"], info["V"]
        if bits & 1:
            raise RuntimeError(f"compute_loca_loss: index {lab} is out of bounds for dimension 2 with size {V} "
                               f"(label at batch {row // L}, position {row % L}; the reference's gather, DT:166)")
        if bits & 2:
            raise RuntimeError(f"student CE: target {lab} is out of bounds (not -100 and not in [0, {V})) "
                               f"at batch {row // L}, position {row % L}")
        for who, e in (("student", serr), ("teacher", terr)):
            if e & 1:
                raise RuntimeError(f"{who} embed_tokens: input id outside the vocabulary")
            if e & 2:
                raise RuntimeError(f"{who}: image-token count does not match the image features "
                                   f"(masked_scatter size mismatch)")


class _KDBase(_Base):
    # subclass hooks
    uses_teacher = True
    ckpt_student_prefix = "student_model."

    def __init__(self, model_name_student, model_name_teacher, processor=None, learning_rate=1e-5, phase=1,
                 seed_teacher: int = 1, seed_student: int = 2, state_dict=None, loss_group_size: int | None = None,
                 accumulate_grad_batches: int | None = None, teacher_fp8: bool | str = False,
                 grad_comm_dtype=None, teacher_residual_f32: bool = False, **_ignored):
        super().__init__()
        self.phase = phase
        self.learning_rate = learning_rate
        self.processor = processor
        self.model_name_student, self.model_name_teacher = model_name_student, model_name_teacher
        # samples whose losses are coupled in one loss call (LoCa's column overrides, NT-Xent
        # negatives).  None = the whole per-rank micro-batch; 1 = the reference's
        # batch_size=1 x accumulate_grad_batches semantics (DT1T:70, :155).
        self.loss_group_size = loss_group_size
        # micro-batches per optimizer step (Lightning's accumulate_grad_batches): only the last
        # backward of a step all-reduces (DP); see also no_sync().  None: the attached
        # Trainer's value (the reference sets it there, DT1T:70, :155), else 1
        self.accumulate_grad_batches = None if accumulate_grad_batches is None else int(accumulate_grad_batches)
        dev = _device()
        # test models draw their weights from the CPU RNG in spec order (bitwise what the
        # reference's fixtures were generated with); the full-size ones from the device RNG
        small = model_name_student not in _HUB_NAMES
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
        # one stream for all student work (forward, backward dgrad chain, AdamW, zero_grad):
        # they are a dependency chain anyway, and HIP multiplexes more streams than hardware
        # queues (GPU_MAX_HW_QUEUES, 4 by default) onto shared queues in enqueue order, which
        # would put the next step's teacher forward behind this step's backward
        self._stu_stream = torch.cuda.Stream(device=dev, priority=STREAM_PRIORITY_HIGH)
        self._opt_stream = self._stu_stream
        self.concurrent_student = True   # False: student forward on the main stream (bench.py --serial)
        self._opt_done = torch.cuda.Event()
        self._opt_pending = False
        # the student backward runs on its own stream, so the next step's teacher forward
        # (main stream; it reads no student state) overlaps it; whatever reads the student
        # gradient or rewrites the saved activations waits for _bwd_done
        self._bwd_stream = self._stu_stream
        self._bwd_done = torch.cuda.Event()
        self._bwd_pending = False
        self.student_model.P.grad_fence = self._grad_fence
        self._ctx = None
        self._errors = _ErrorWatch(dev)
        self._errors.bind(self.student_model, self.teacher_model)
        self.keep_logits = False         # tests: keep the step's logits in last_logits
        # fuse_row_stats: the lm_head epilogues emit the KD loss's row statistics.  Off by default:
        # measured slower (profiles/r03/row_stats_fusion_ab.txt); tests / tools set the attribute
        self.fuse_row_stats = False
        # the student's row statistics on the student stream ahead of the loss (kd_loss_student_stats;
        # False leaves them in the loss's own pass, for A/B)
        self.student_stats_early = True
        # kd_loss_params.standin_count: partner partials the register-resident LoCa kernel recomputed
        # (its fallback when a row's slices are not co-resident; bench.py reports it)
        self.loss_standins = torch.zeros(1, dtype=torch.int32, device=dev)
        self.last_terms = None
        self.last_ntxent = None
        self.last_logits = None
        self.last_post = None            # (student, teacher) post-LN hook outputs when keep_logits
        self._micro = 0                  # backward passes since the last optimizer step
        self._no_sync_depth = 0
        # data parallel
        import torch.distributed as dist
        self._dist = dist if (dist.is_available() and dist.is_initialized()) else None
        self._gsync = None
        self._marks = None               # BackwardMarks of the student layout (first callback)
        if self._dist is not None:
            if self.uses_teacher:
                # teacher weights broadcast once from rank 0, then read-only in every GPU's HBM
                self._dist.broadcast(self.teacher_model.P.flat, src=0)
            self._dist.broadcast(self.student_model.P.flat, src=0)
            self.student_model.P.master.copy_(self.student_model.P.flat.float())
            # grad_comm_dtype=torch.bfloat16: bf16 all-reduce buckets (half the xGMI bytes; dp.py)
            self._gsync = GradSync(self._dist, self.student_model.P.grad, comm_dtype=grad_comm_dtype)
        # fp8 (e4m3) teacher weights, quantised once after the broadcast (BASELINE config c4;
        # the reference loads the teacher fp16, DT:43-48)
        # teacher_fp8: False, True (= "all") or a modeling.FP8_FAMILIES policy name ("lm", "lm_mlp", ...)
        # teacher_residual_f32: the teacher's 3584-wide Qwen2 residual stream in fp32 as well (the
        # c1 reference teacher runs fp32 end to end, LB:29-33; default bf16)
        self.teacher_residual_f32 = bool(teacher_residual_f32)
        if self.teacher_residual_f32 and self.teacher_model is not None:
            self.teacher_model.set_lm_stream_f32(True)
        if teacher_fp8 is True:
            teacher_fp8 = "all"
        self.teacher_fp8 = teacher_fp8 if (teacher_fp8 and self.teacher_model is not None) else False
        if self.teacher_fp8:
            self.teacher_model.enable_fp8(self.teacher_fp8)

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

    def _trainer_precision(self):
        try:
            tr = self.trainer   # LightningModule.trainer raises when no Trainer is attached
        except Exception:
            tr = None
        return getattr(tr, "precision", None) if tr is not None else None

    def setup(self, stage=None):                         # DT:88-91
        check_trainer_precision(self._trainer_precision())

    # --------------------------------------------------------------- losses ----
    def _loss_spec(self):
        """(kd variant, T, kd_weight, ce_weight, ntxent weight or None)."""
        raise NotImplementedError

    def configure_optimizers(self):                      # DT:198-201
        check_trainer_precision(self._trainer_precision())
        opt = FusedAdamW(self, lr=self.learning_rate)
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
        return [opt], [sched]

    # ------------------------------------------------------------- the step ----
    def _teacher_forward(self, batch, need_feats, row_stats=None):
        tfwd = self.teacher_model.forward(batch["rgb_input_ids"], batch["rgb_pixel_values"], batch["image_sizes"],
                                          save=False, want_post_ln=need_feats, want_logits=True, row_stats=row_stats)
        return tfwd["logits"], tfwd.get("post_ln"), tfwd.get("row_stats")

    def _groups(self, B):
        G = self.loss_group_size or B
        if G <= 0 or B % G:
            raise ValueError(f"loss_group_size {G} must divide the per-rank batch {B}")
        return G, B // G

    def forward(self, batch, train: bool = False):
        """The reference's forward(batch) (DT:206-271): total loss as a 0-d fp32 tensor."""
        variant, T, kd_w, ce_w, ctr_w = self._loss_spec()
        labels = batch["labels"]
        image_sizes = batch["image_sizes"]
        B, L = batch["depth_input_ids"].shape
        G, ng = self._groups(B)
        need_feats = ctr_w is not None
        main = torch.cuda.current_stream()
        s = self.student_model
        # student forward on its own stream beside the teacher forward. It first waits for
        # everything already queued on the main stream (so caching-allocator blocks the
        # previous step freed there are reusable) and for the previous optimizer step (the
        # student weights); the main stream joins it before the loss. The teacher (the long
        # pole, large GEMMs that do not read student weights) is ENQUEUED first.
        side = self._stu_stream if self.concurrent_student else main
        side.wait_stream(main)
        if self._bwd_pending:     # the saved activations of the last backward are rewritten
            side.wait_event(self._bwd_done)
        if self._opt_pending:
            side.wait_event(self._opt_done)
            self._opt_pending = False
        # the lm_head epilogues emit the loss's per-row softmax statistics (kd_gemm_desc.row_stats)
        # so the loss does not read both logit tensors once more just for them (fuse_row_stats;
        # default: the loss's own pass)
        Vs_ = s.cfg.text.vocab
        fuse = self.fuse_row_stats
        t_logits = t_post = t_rst = None
        if self.uses_teacher:
            t_logits, t_post, t_rst = self._teacher_forward(batch, need_feats,
                                                            (Vs_, 1.0 / T, True) if fuse else None)
        with torch.cuda.stream(side):
            sfwd = s.forward(batch["depth_input_ids"], batch["depth_pixel_values"], image_sizes, save=train,
                             want_post_ln=need_feats, want_logits=True, row_stats=(Vs_, 1.0 / T, False) if fuse else None)
            s_logits = sfwd.pop("logits")
            s_rst = sfwd.pop("row_stats", None)
            # the student half of the loss's row statistics, on the student stream right after its
            # lm_head: it finishes before the teacher forward (c1: ~7 ms of slack), so the loss,
            # the one stretch of the step with nothing beside it, reads only the teacher's logits
            # for its statistics (kd_loss_params.s_stats; bit-identical)
            s_st = None
            if s_rst is None and self.uses_teacher and self.student_stats_early:
                s_st = ops.kd_loss_student_stats(s_logits, temperature=T)
                s_st.record_stream(main)   # read by the loss on the caller's stream
        main.wait_stream(side)
        Vs = s_logits.shape[1]
        s3 = s_logits.view(B, L, Vs)
        t3 = None if t_logits is None else t_logits.view(B, L, -1)
        loss4 = torch.empty(4, dtype=torch.float32, device=s_logits.device)
        dlogits = torch.empty((B, L, Vs), dtype=torch.bfloat16, device=s_logits.device) if train else None
        # dlogits are stored relative to the CE coefficient (kd_loss_params.dscale): the one-hot
        # element of every row is then ~ -1, exact in bf16, instead of the same bf16-rounded
        # -1/n_valid in every row, a systematic +0.13 % on the whole gradient (tools/grad_bias_study.py)
        dscale = torch.empty(1, dtype=torch.float32, device=s_logits.device) if train else None
        if s_rst is not None and t3 is not None and t_rst is None:
            s_rst = None   # both or neither
        rs = slice(0, 0)
        for g in range(ng):   # loss groups: mean over groups of each group's loss
            sl = slice(g * G, (g + 1) * G)
            rs = slice(g * G * L, (g + 1) * G * L)
            ops.kd_loss_fwd_bwd(s3[sl], None if t3 is None else t3[sl], labels[sl], variant,
                                temperature=T, alpha=0.8, kd_weight=kd_w, ce_weight=ce_w, grad_scale=1.0 / ng,
                                want_grad=train, loss_out=loss4, out_scale=1.0 / ng, accumulate=g > 0,
                                dlogits_out=None if dlogits is None else dlogits[sl], err_out=self._errors.kd,
                                row_base=g * G * L, dscale=dscale, dscale_given=g > 0,
                                s_row_stats=None if s_rst is None else s_rst[rs],
                                t_row_stats=None if (s_rst is None or t_rst is None) else t_rst[rs],
                                s_stats=None if s_st is None else s_st[rs], standin_count=self.loss_standins)
        del s_rst, t_rst, s_st
        if self.keep_logits:
            self.last_logits = (s3, t3)
            self.last_post = (sfwd.get("post_ln"), t_post)
        del s_logits, t_logits, s3, t3
        total = loss4[3]
        dps = None
        if need_feats:
            NP = s.cfg.vision.n_patches
            NI = sfwd["post_ln"].shape[0] // NP                      # the batch's real tiles (KAT 7: 2B at 336x336)
            ps = ops.row_group_mean(sfwd["post_ln"], NI, NP)        # DT:243-244
            pt = ops.row_group_mean(t_post, NI, NP)
            cum = [0]
            for n in sfwd["tile_counts"]:                            # pooled tile rows of each sample
                cum.append(cum[-1] + n)
            ntx_rows = torch.empty((ng, 2), dtype=torch.float32, device=ps.device)
            dps = torch.empty_like(ps) if train else None
            for g in range(ng):                                      # DT:393-416 per group
                r = slice(cum[g * G], cum[(g + 1) * G])
                ops.ntxent(ps[r], pt[r], tau=0.07, weight=ctr_w / ng, want_grad=train, loss_out=ntx_rows[g],
                           dfs_out=None if dps is None else dps[r])
            ntx = ntx_rows.sum(0) if ng > 1 else ntx_rows[0]
            total = total + ntx[0]
            self.last_ntxent = (ntx[0], ntx_rows[:, 1].mean() if ng > 1 else ntx_rows[0, 1])
        self.last_terms = loss4
        self._errors.record(dict(L=L, V=Vs))
        if train:
            self._ctx = dict(sfwd=sfwd, dlogits=dlogits, dscale=dscale, dps=dps)
        return total

    def _grad_fence(self):
        if self._bwd_pending:
            torch.cuda.current_stream().wait_event(self._bwd_done)
        if self._gsync is not None and self._gsync.works:
            self._gsync.wait()   # reading .grad after backward sees the reduced gradient (DDP)

    def _backward(self, gscale):
        ctx, self._ctx = self._ctx, None
        main = torch.cuda.current_stream()
        bwd = self._bwd_stream if self.concurrent_student else main
        if bwd is not main:
            bwd.wait_stream(main)
            sf = ctx["sfwd"]
            for t in (gscale, ctx["dlogits"], ctx["dscale"], ctx["dps"], sf["hn"], sf["src"], sf["ids"],
                      sf.get("post_ln")):
                if t is not None:
                    t.record_stream(bwd)   # freed on the host before the backward has run
        with torch.cuda.stream(bwd):
            self._backward_body(ctx, gscale)
        self._bwd_done.record(bwd)
        self._bwd_pending = bwd is not main

    def _backward_body(self, ctx, gscale):
        s = self.student_model
        self._micro += 1
        sync = self._gsync is not None and self._no_sync_depth == 0 and \
            self._micro % self._accumulate() == 0
        if self._gsync is not None:
            self._gsync.begin(sync, top=self._trainable_range()[1])
        sf = ctx["sfwd"]
        hn = sf["hn"]
        W = s.lm_head_weight()
        dl = ctx["dlogits"].view(hn.shape[0], -1)
        dscale = ops.scalar_mul(gscale, ctx["dscale"])                      # upstream x the dlogits scale
        dhn = ops.gemm(dl, W.t(), alpha_dev=dscale)                          # lm_head dgrad
        if s.train_language:   # lm_head / tied embed wgrad, on the lane ahead of the runtime's backward
            s.wlane.run(lambda: ops.gemm(dl.t(), hn.t(), out=s.lm_head_grad(), accumulate=True, alpha_dev=dscale),
                        dl, hn, dscale)
        del dl, ctx["dlogits"]
        dpost = None
        if ctx["dps"] is not None and s.train_vision:
            # the gradient of each tile's pooled feature, fp32 (kd_model_backward spreads it over the
            # tile's rows without a bf16 rounding: tools/ntx_bias_study.py)
            dpost = ops.scale_f32(ctx["dps"], gscale)
        s.backward(sf, dhn, dpost, on_layer_done=self._on_layer_done if sync else None)
        if self._gsync is not None:
            self._gsync.end(*self._trainable_range())

    def _accumulate(self) -> int:
        """Micro-batches per optimizer step: the constructor's value, else the attached
        Lightning Trainer's accumulate_grad_batches, else 1."""
        if self.accumulate_grad_batches is not None:
            return max(1, self.accumulate_grad_batches)
        try:
            tr = self.trainer   # LightningModule.trainer raises when no Trainer is attached
        except Exception:
            tr = None
        return max(1, int(getattr(tr, "accumulate_grad_batches", 1) or 1)) if tr is not None else 1

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes inside the block accumulate locally without the DP all-reduce
        (DDP no_sync); the optimizer step reduces whatever is left unsynced."""
        self._no_sync_depth += 1
        try:
            yield
        finally:
            self._no_sync_depth -= 1

    # ------------------------------------------------------- data parallel ----
    def _on_layer_done(self, code):
        """Bucketed all-reduce of the student grads as soon as the backward has made them final
        (kd_model_backward's callback, include/kdstep.h ABI 9).

        Flat layout [vision | projector | embed, layers 0..N-1, norm(, lm_head)]; the backward
        finishes the tail first (lm_head, norm), then layers N-1..0 (code = the layer), then
        embed / projector (KD_CB_EMBED_PROJECTOR), then the SigLIP layers top-down
        (KD_CB_VISION_LAYER(i)), the patch / position embeddings last (GradSync.end).
        Everything from the part's first parameter to the high-water mark is final."""
        s = self.student_model
        if self._marks is None:
            self._marks = BackwardMarks(s.P.offsets)
        first = self._marks.first(code, s.train_language, s.train_projector, s.train_vision)
        if first is None:
            return
        lane = getattr(s, "wlane", None)
        self._gsync.layer_done(first, before_launch=lane.join if lane is not None else None)

    def _check_errors(self, block: bool):
        self._errors.check(block=block)

    def check_errors(self):
        """Wait for every queued step and raise its device-detected error (label range,
        token ids, image-token count), if any."""
        self._errors.check(block=True)

    # ---------------------------------------------------------- Lightning API ----
    def training_step(self, batch, batch_idx):           # DT:123-131
        self._check_errors(block=False)
        total = self.forward(batch, train=True)
        loss = _KDStepFn.apply(self._anchor, total, self)
        self.log("train_loss", loss, on_step=True, on_epoch=True, prog_bar=True, logger=True)
        return loss

    def validation_step(self, batch, batch_idx):         # DT:133-138
        with torch.no_grad():
            loss = self.forward(batch, train=False)
        self._check_errors(block=True)
        self.log("val_loss", loss, on_step=False, on_epoch=True, prog_bar=True, logger=True)
        return loss

    # ------------------------------------------------------------ checkpoints ----
    def kd_state_dict(self):
        if self._opt_pending:   # weights of a queued optimizer step
            torch.cuda.current_stream().wait_event(self._opt_done)
        sd = {f"{self.ckpt_student_prefix}{k}": v for k, v in self.student_model.P.state_dict().items()}
        if self.teacher_model is not None:
            sd.update({f"teacher_model.{k}": v for k, v in self.teacher_model.P.state_dict().items()})
        return sd

    def load_kd_state_dict(self, sd):
        self.student_model.P.load_state_dict(sd, prefix=self.ckpt_student_prefix)
        if self.teacher_model is not None and any(k.startswith("teacher_model.") for k in sd):
            self.teacher_model.P.load_state_dict(sd, prefix="teacher_model.")
            if getattr(self.teacher_model, "fp8", False):
                self.teacher_model.enable_fp8(self.teacher_model.fp8_families)   # re-quantise the new weights

    def load_hf_weights(self, student: dict | None = None, teacher: dict | None = None, strict: bool = True):
        """The weights `from_pretrained(model_name_*)` would load (DT:33-48), given as
        LlavaOnevisionForConditionalGeneration state_dicts in the transformers-4.45 or 5.x
        key layout (e.g. read from the hub's safetensors files with safetensors.torch.load_file)."""
        if student is not None:
            self.student_model.load_hf_state_dict(student, strict=strict)
        if teacher is not None:
            if self.teacher_model is None:
                raise ValueError(f"{type(self).__name__} has no teacher")
            self.teacher_model.load_hf_state_dict(teacher, strict=strict)

    def _hparams(self):
        # everything that changes the objective or the update is saved, so load_from_checkpoint
        # resumes the same run (loss grouping changes the loss: test_loss_group_size_*)
        return {"model_name_student": self.model_name_student, "model_name_teacher": self.model_name_teacher,
                "learning_rate": self.learning_rate, "phase": self.phase, **self._run_hparams()}

    def _run_hparams(self):
        return {"loss_group_size": self.loss_group_size, "accumulate_grad_batches": self.accumulate_grad_batches,
                "teacher_fp8": getattr(self, "teacher_fp8", False),
                "teacher_residual_f32": getattr(self, "teacher_residual_f32", False)}

    def on_train_epoch_end(self):
        """A batch rejected among the last steps of an epoch is reported here (the reference
        raises inside its training_step, DT:166), not silently dropped."""
        self.check_errors()

    def on_train_end(self):
        self.check_errors()

    def save_checkpoint(self, path, epoch: int = 0, global_step: int = 0):
        """Lightning-style .ckpt: {'state_dict': {student_model.*, teacher_model.*}, ...}."""
        self.check_errors()   # never write weights past an unreported rejected batch
        sd = {k: v.detach().cpu() for k, v in self.kd_state_dict().items()}
        torch.save({"state_dict": sd, "epoch": epoch, "global_step": global_step,
                    "pytorch-lightning_version": "2.4.0", "hyper_parameters": self._hparams()}, path)

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location=None, **kw):
        """LightningModule.load_from_checkpoint: the constructor arguments come from the
        keywords given here (the reference passes model names, processor, torch_dtype,
        map_location, phase: evaluate_onevision.py:65-73, BDT:86-91), falling back to the
        checkpoint's saved hyper-parameters; then the state_dict is loaded."""
        ck = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        hp = dict(ck.get("hyper_parameters", {}))
        sig = inspect.signature(cls.__init__)
        args = {}
        var_kw = False
        for name, prm in list(sig.parameters.items())[1:]:
            if prm.kind == prm.VAR_KEYWORD:
                var_kw = True
            if prm.kind in (prm.VAR_KEYWORD, prm.VAR_POSITIONAL):
                continue
            if name in kw:
                args[name] = kw.pop(name)
            elif name in hp:
                args[name] = hp[name]
        if var_kw:   # the saved run knobs a subclass forwards to _KDBase through **kw
            for name in ("loss_group_size", "accumulate_grad_batches", "teacher_fp8", "teacher_residual_f32"):
                if name in hp and name not in args and name not in kw:
                    args[name] = hp[name]
        kw.pop("torch_dtype", None)   # the build's weights are bf16 in HBM whatever the caller's dtype
        return cls(**args, state_dict=ck["state_dict"], **kw)


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
        check_trainer_precision(self._trainer_precision())
        return FusedAdamW(self, lr=self.learning_rate)


class LlavaOnevisionModule(_KDBase):
    """Depth-student SFT baseline (BD:6-138): loss = the student's CE only.  Its Lightning
    checkpoint holds the student under `model.*` (the reference's attribute, BD:15)."""
    uses_teacher = False
    ckpt_student_prefix = "model."

    def __init__(self, model_name, processor=None, learning_rate=2e-5, **kw):
        super().__init__(model_name, None, processor, learning_rate, phase=0, **kw)
        self.model_name = model_name
        self.model = self.student_model

    def _hparams(self):
        return {"model_name": self.model_name, "learning_rate": self.learning_rate, **self._run_hparams()}

    def _loss_spec(self):
        return "none", 1.0, 0.0, 1.0, None

    def configure_optimizers(self):        # BD:137-138
        check_trainer_precision(self._trainer_precision())
        return FusedAdamW(self, lr=self.learning_rate)
