"""LLaVA-OneVision (SigLIP + projector + anyres pack + Qwen2 + lm_head) on the HIP kernels.

The reference loads `LlavaOnevisionForConditionalGeneration` from transformers (DT:33-48)
and calls it as `model(input_ids=, pixel_values=, labels=, image_sizes=)` (DT:228, :238).
This module is the build's own implementation of that forward and of its autograd
backward, written as an explicit layer-by-layer forward (saving what the backward needs)
and a hand-ordered backward; every FLOP runs in libkdstep.so (ops.py).  PyTorch only
allocates tensors.

Parameters live in ONE flat bf16 buffer (plus flat fp32 master / grad / Adam buffers for
a trainable model) in the transformers-4.45 state_dict order and names
(`vision_tower.vision_model.*`, `multi_modal_projector.*`, `image_newline`,
`language_model.model.*`, `language_model.lm_head.weight`), so:
  - the fused q|k|v and gate|up weights are contiguous views (no concatenation copies),
  - every freeze mask of the reference (DT:468-523) is a contiguous range -> one AdamW
    launch and one bucketed all-reduce range,
  - checkpoints keep the reference's key layout.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import anyres
from . import ops

IMAGE_TOKEN_ID = 151646


# ------------------------------------------------------------------ configs ----
@dataclass(frozen=True)
class VisionConfig:
    hidden: int = 1152
    inter: int = 4304
    layers: int = 26
    heads: int = 16
    patch: int = 14
    image: int = 384
    eps: float = 1e-6

    @property
    def hd(self):
        return self.hidden // self.heads

    @property
    def hdp(self):  # attention kernel head-dim padding
        return 64 if self.hd <= 64 else (96 if self.hd <= 80 else 128)

    @property
    def grid(self):
        return self.image // self.patch

    @property
    def n_patches(self):
        return self.grid * self.grid

    @property
    def kpatch(self):  # im2col K padded to a multiple of 8 (588 -> 592)
        k = 3 * self.patch * self.patch
        return (k + 7) // 8 * 8


@dataclass(frozen=True)
class TextConfig:
    hidden: int
    inter: int
    layers: int
    heads: int
    kv_heads: int
    head_dim: int
    vocab: int
    tie: bool = False
    rope_theta: float = 1e6
    eps: float = 1e-6


@dataclass(frozen=True)
class LlavaConfig:
    vision: VisionConfig
    text: TextConfig
    image_token_id: int = IMAGE_TOKEN_ID
    projector_act: str = "gelu_erf"   # projector_hidden_act "gelu" (exact erf)


# llava-hf/llava-onevision-qwen2-{7b,0.5b}-ov-hf (public configs; the reference only names them, DT1T:76-78)
TEACHER_7B = LlavaConfig(VisionConfig(), TextConfig(3584, 18944, 28, 28, 4, 128, 152064, tie=False))
STUDENT_05B = LlavaConfig(VisionConfig(), TextConfig(896, 4864, 24, 14, 2, 64, 151936, tie=True))


def tiny_config(teacher: bool = False) -> LlavaConfig:
    """Reduced-depth/width configs at the REAL vocab and real 336^2 token layout (tests)."""
    v = VisionConfig(hidden=64, inter=128, layers=2, heads=2)
    if teacher:
        t = TextConfig(hidden=128, inter=256, layers=2, heads=2, kv_heads=1, head_dim=64, vocab=152064, tie=False)
    else:
        t = TextConfig(hidden=128, inter=192, layers=2, heads=2, kv_heads=1, head_dim=64, vocab=151936, tie=True)
    return LlavaConfig(v, t)


# -------------------------------------------------------------- param specs ----
@dataclass
class Spec:
    name: str                 # transformers-4.45 state_dict key
    shape: tuple              # storage shape in the flat buffer
    init: str = "normal"      # normal | ones | zeros | patch
    ckpt_shape: tuple | None = None   # shape in the checkpoint when it differs


def param_specs(cfg: LlavaConfig) -> list[Spec]:
    V, T = cfg.vision, cfg.text
    S: list[Spec] = []
    vp = "vision_tower.vision_model."
    S.append(Spec(vp + "embeddings.patch_embedding.weight", (V.hidden, V.kpatch), "patch",
                  ckpt_shape=(V.hidden, 3, V.patch, V.patch)))
    S.append(Spec(vp + "embeddings.patch_embedding.bias", (V.hidden,), "zeros"))
    S.append(Spec(vp + "embeddings.position_embedding.weight", (V.n_patches, V.hidden)))
    for i in range(V.layers):
        p = f"{vp}encoder.layers.{i}."
        for n in ("q", "k", "v"):     # contiguous: fused qkv weight [3D, D]
            S.append(Spec(p + f"self_attn.{n}_proj.weight", (V.hidden, V.hidden)))
        for n in ("q", "k", "v"):     # fused qkv bias [3D]
            S.append(Spec(p + f"self_attn.{n}_proj.bias", (V.hidden,), "zeros"))
        S.append(Spec(p + "self_attn.out_proj.weight", (V.hidden, V.hidden)))
        S.append(Spec(p + "self_attn.out_proj.bias", (V.hidden,), "zeros"))
        S.append(Spec(p + "layer_norm1.weight", (V.hidden,), "ones"))
        S.append(Spec(p + "layer_norm1.bias", (V.hidden,), "zeros"))
        S.append(Spec(p + "mlp.fc1.weight", (V.inter, V.hidden)))
        S.append(Spec(p + "mlp.fc1.bias", (V.inter,), "zeros"))
        S.append(Spec(p + "mlp.fc2.weight", (V.hidden, V.inter)))
        S.append(Spec(p + "mlp.fc2.bias", (V.hidden,), "zeros"))
        S.append(Spec(p + "layer_norm2.weight", (V.hidden,), "ones"))
        S.append(Spec(p + "layer_norm2.bias", (V.hidden,), "zeros"))
    S.append(Spec(vp + "post_layernorm.weight", (V.hidden,), "ones"))
    S.append(Spec(vp + "post_layernorm.bias", (V.hidden,), "zeros"))
    S.append(Spec("multi_modal_projector.linear_1.weight", (T.hidden, V.hidden)))
    S.append(Spec("multi_modal_projector.linear_1.bias", (T.hidden,), "zeros"))
    S.append(Spec("multi_modal_projector.linear_2.weight", (T.hidden, T.hidden)))
    S.append(Spec("multi_modal_projector.linear_2.bias", (T.hidden,), "zeros"))
    S.append(Spec("image_newline", (T.hidden,)))
    lp = "language_model.model."
    S.append(Spec(lp + "embed_tokens.weight", (T.vocab, T.hidden)))
    qd, kd = T.heads * T.head_dim, T.kv_heads * T.head_dim
    for i in range(T.layers):
        p = f"{lp}layers.{i}."
        S.append(Spec(p + "self_attn.q_proj.weight", (qd, T.hidden)))
        S.append(Spec(p + "self_attn.k_proj.weight", (kd, T.hidden)))
        S.append(Spec(p + "self_attn.v_proj.weight", (kd, T.hidden)))
        S.append(Spec(p + "self_attn.q_proj.bias", (qd,), "zeros"))
        S.append(Spec(p + "self_attn.k_proj.bias", (kd,), "zeros"))
        S.append(Spec(p + "self_attn.v_proj.bias", (kd,), "zeros"))
        S.append(Spec(p + "self_attn.o_proj.weight", (T.hidden, qd)))
        S.append(Spec(p + "mlp.gate_proj.weight", (T.inter, T.hidden)))
        S.append(Spec(p + "mlp.up_proj.weight", (T.inter, T.hidden)))
        S.append(Spec(p + "mlp.down_proj.weight", (T.hidden, T.inter)))
        S.append(Spec(p + "input_layernorm.weight", (T.hidden,), "ones"))
        S.append(Spec(p + "post_attention_layernorm.weight", (T.hidden,), "ones"))
    S.append(Spec(lp + "norm.weight", (T.hidden,), "ones"))
    if not T.tie:
        S.append(Spec("language_model.lm_head.weight", (T.vocab, T.hidden)))
    return S


# ---------------------------------------------------------------- the store ----
class ParamStore:
    """All parameters of one model as views of flat buffers (see module docstring)."""

    def __init__(self, cfg: LlavaConfig, device, trainable: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        self.specs = param_specs(cfg)
        self.offsets: dict[str, tuple[int, int]] = {}
        off = 0
        for s in self.specs:
            n = int(np.prod(s.shape))
            off = (off + 7) // 8 * 8     # 16-B alignment of every view
            self.offsets[s.name] = (off, n)
            off += n
        self.numel = (off + 7) // 8 * 8
        self.flat = torch.zeros(self.numel, dtype=torch.bfloat16, device=self.device)
        self.trainable = trainable
        if trainable:
            self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            self.exp_avg = torch.zeros_like(self.master)
            self.exp_avg_sq = torch.zeros_like(self.master)
        self._views = {s.name: self.view(s.name) for s in self.specs}
        # region boundaries of the freeze masks (DT:468-523)
        first_proj = self.offsets["multi_modal_projector.linear_1.weight"][0]
        first_lm = self.offsets["language_model.model.embed_tokens.weight"][0]
        self.regions = {"vision": (0, first_proj), "projector": (first_proj, first_lm),
                        "language": (first_lm, self.numel)}

    # -- views
    def view(self, name, buf=None):
        off, n = self.offsets[name]
        shape = next(s.shape for s in self.specs if s.name == name)
        return (self.flat if buf is None else buf)[off:off + n].view(shape)

    def __getitem__(self, name):
        return self._views[name]

    def span(self, first: str, last: str, rows: int, cols: int, buf=None):
        """A contiguous 2-D view from param `first` through `last` (fused q|k|v, gate|up)."""
        o0, _ = self.offsets[first]
        o1, n1 = self.offsets[last]
        if (o1 + n1 - o0) != rows * cols:
            raise RuntimeError(f"span {first}..{last} is not contiguous")
        return (self.flat if buf is None else buf)[o0:o1 + n1].view(rows, cols)

    def grad_view(self, name):
        return self.view(name, self.grad)

    def grad_span(self, first, last, rows, cols):
        return self.span(first, last, rows, cols, self.grad)

    # -- initialisation (synthetic: no checkpoints are reachable offline)
    def init_(self, seed: int, std: float = 0.02, cpu_rng: bool = False):
        """Seeded N(0, std) weights, ones for norm weights, zeros for biases.

        cpu_rng=True draws every tensor from a CPU torch.Generator in spec order (bitwise
        reproducible by the CPU oracle); otherwise the device RNG is used (big models)."""
        g = torch.Generator(device="cpu" if cpu_rng else self.device).manual_seed(seed)
        for s in self.specs:
            v = self[s.name]
            if s.init == "ones":
                v.fill_(1.0)
            elif s.init == "zeros":
                v.zero_()
            else:
                shape = s.ckpt_shape if s.init == "patch" else s.shape
                w = torch.randn(shape, generator=g, device="cpu" if cpu_rng else self.device) * std
                if s.init == "patch":
                    v.zero_()
                    v[:, :w[0].numel()] = w.reshape(shape[0], -1).to(self.device, torch.bfloat16)
                else:
                    v.copy_(w.to(self.device, torch.bfloat16))
        if self.trainable:
            self.master.copy_(self.flat.float())

    # -- checkpoint layout (transformers-4.45 names)
    def state_dict(self, prefix: str = "") -> dict:
        out = {}
        for s in self.specs:
            t = self[s.name]
            if s.ckpt_shape is not None:
                k = int(np.prod(s.ckpt_shape[1:]))
                t = t[:, :k].reshape(s.ckpt_shape)
            out[prefix + s.name] = t
        if self.cfg.text.tie:
            out[prefix + "language_model.lm_head.weight"] = self["language_model.model.embed_tokens.weight"]
        return out

    def load_state_dict(self, sd: dict, prefix: str = "", strict: bool = True):
        seen = set()
        for s in self.specs:
            key = prefix + s.name
            if key not in sd:
                if strict:
                    raise KeyError(f"missing key {key}")
                continue
            t = sd[key].to(self.device)
            v = self[s.name]
            if s.ckpt_shape is not None:
                v.zero_()
                v[:, :int(np.prod(s.ckpt_shape[1:]))] = t.reshape(s.ckpt_shape[0], -1).to(torch.bfloat16)
            else:
                v.copy_(t.to(torch.bfloat16).view(v.shape))
            seen.add(key)
        if self.trainable:
            self.master.copy_(self.flat.float())
        return seen


# ------------------------------------------------------------------ helpers ----
def rope_tables(seq: int, hd: int, theta: float, device):
    """cos/sin [seq, hd/2] fp32 as HF's Qwen2RotaryEmbedding (inv_freq in fp32)."""
    inv = (1.0 / (theta ** (np.arange(0, hd, 2, dtype=np.int64).astype(np.float32) / hd))).astype(np.float32)
    f = np.arange(seq, dtype=np.float32)[:, None] * inv[None, :]
    return (torch.from_numpy(np.cos(f).astype(np.float32)).to(device),
            torch.from_numpy(np.sin(f).astype(np.float32)).to(device))


class Saved(dict):
    """Per-layer activations kept for the backward."""


# priority of the training step's streams (lower = higher; 0 = default); the teacher
# prefetch stream stays at 0 (KD_STREAM_PRIORITY=0 turns the distinction off)
STREAM_PRIORITY_HIGH = int(os.environ.get("KD_STREAM_PRIORITY", "-1"))


class WgradLane:
    """Weight-gradient work (dW GEMMs, bias column sums) on a side stream.

    A linear layer's dW = dY^T X feeds only the optimizer, so it runs beside the dgrad
    chain dX = dY W that the next layer waits for; the student's backward GEMMs (hidden
    896, SigLIP 1152) fill 100-230 tiles of 256x256, fewer than the 256 CUs, so the two
    streams fill each other's idle CUs.  `run` orders the side stream after everything
    queued on the current stream, keeps its operands' memory alive for it (record_stream)
    and returns an event the current stream waits on before it updates an operand in place;
    `join` makes the current stream wait for all of it (before grads are read)."""

    def __init__(self, device):
        self.stream = torch.cuda.Stream(device=device, priority=STREAM_PRIORITY_HIGH)
        # split-K default for the lane's GEMMs (0 = the library's cost model, which prices a
        # GEMM as if it had the GPU to itself; 1 = never split: beside the dgrad chain an
        # unsplit 76-150-tile dW GEMM leaves the other CUs to it and skips the fp32
        # partial-plane round trip)
        self.split_k = int(os.environ.get("KD_WGRAD_SPLIT_K", "0"))

    def run(self, fn, *keep):
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream), ops.gemm_split_default(self.split_k):
            fn()
        for t in keep:
            if t is not None:
                t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    def join(self):
        torch.cuda.current_stream().wait_stream(self.stream)


def _wait(ev):
    if ev is not None:
        torch.cuda.current_stream().wait_event(ev)


# --------------------------------------------------------------------- model ----
class LlavaOnevisionModel:
    """One LLaVA-OneVision instance (teacher or student) on a ParamStore."""

    def __init__(self, cfg: LlavaConfig, device, trainable: bool = False, seed: int | None = None,
                 cpu_rng: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        self.P = ParamStore(cfg, device, trainable)
        if seed is not None:
            self.P.init_(seed, cpu_rng=cpu_rng)
        self._rope = {}
        self._maps = {}
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        # which regions receive weight gradients (freeze masks, DT:468-523)
        self.train_vision = self.train_projector = self.train_language = trainable
        self.wlane = WgradLane(self.device) if (trainable and self.device.type == "cuda") else None
        self.tied_grad_event = None   # lm_head wgrad into the tied embedding grad (kd_module._backward)

    # -- freeze helpers mirroring DT:468-523 (applied to the student)
    def set_trainable(self, vision: bool, projector: bool, language: bool):
        self.train_vision, self.train_projector, self.train_language = vision, projector, language

    def _rope_for(self, L):
        if L not in self._rope:
            self._rope[L] = rope_tables(L, self.cfg.text.head_dim, self.cfg.text.rope_theta, self.device)
        return self._rope[L]

    def _src_map(self, input_ids, image_sizes, tiles):
        key = (tuple(tuple(int(v) for v in hw) for hw in image_sizes), tiles)
        if key not in self._maps:
            maps, lens = anyres.batch_maps(key[0], tiles)
            w = max(lens)
            arr = np.full((len(maps), w), -2, dtype=np.int32)
            for i, m in enumerate(maps):
                arr[i, :len(m)] = m
            self._maps[key] = (torch.from_numpy(arr).to(self.device), torch.tensor(lens, dtype=torch.int32,
                                                                                      device=self.device))
        maps, lens = self._maps[key]
        return ops.image_src_map(input_ids, self.cfg.image_token_id, maps, lens, self.err)

    # ============================================================== vision ====
    def vision_forward(self, pixels, save: bool):
        """pixels [NI, 3, 384, 384] -> (x_last [NT, D] pre-post-LN, post_ln [NT, D], saves)."""
        V, P = self.cfg.vision, self.P
        NI = pixels.shape[0]
        NT = NI * V.n_patches
        vp = "vision_tower.vision_model."
        rows = ops.patchify(pixels, V.patch, V.kpatch)                           # [NT, Kp]
        x = ops.gemm(rows, P[vp + "embeddings.patch_embedding.weight"],
                     bias=P[vp + "embeddings.patch_embedding.bias"],
                     residual=P[vp + "embeddings.position_embedding.weight"], residual_row_mod=V.n_patches)
        saved = [rows] if save else None
        layers = []
        D = V.hidden
        for i in range(V.layers):
            p = f"{vp}encoder.layers.{i}."
            Wqkv = P.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight", 3 * D, D)
            bqkv = P.span(p + "self_attn.q_proj.bias", p + "self_attn.v_proj.bias", 1, 3 * D).view(-1)
            h, m1, r1 = ops.norm_fwd(x, P[p + "layer_norm1.weight"], P[p + "layer_norm1.bias"], V.eps, save_stats=save)
            qkv = ops.gemm(h, Wqkv, bias=bqkv)
            q, k, v = ops.qkv_split(qkv, NI, V.n_patches, V.heads, V.heads, V.hd, V.hdp)
            del qkv
            o, lse = ops.attn_fwd(q, k, v, V.hd, causal=False, want_lse=save)
            o2 = o.view(NT, D)
            x_mid = ops.gemm(o2, P[p + "self_attn.out_proj.weight"], bias=P[p + "self_attn.out_proj.bias"], residual=x)
            h2, m2, r2 = ops.norm_fwd(x_mid, P[p + "layer_norm2.weight"], P[p + "layer_norm2.bias"], V.eps,
                                      save_stats=save)
            pre = torch.empty((NT, V.inter), dtype=torch.bfloat16, device=self.device) if save else None
            u = ops.gemm(h2, P[p + "mlp.fc1.weight"], bias=P[p + "mlp.fc1.bias"], act="gelu_tanh", aux=pre)
            x_out = ops.gemm(u, P[p + "mlp.fc2.weight"], bias=P[p + "mlp.fc2.bias"], residual=x_mid)
            if save:
                layers.append(Saved(x=x, h=h, m1=m1, r1=r1, q=q, k=k, v=v, o=o2, lse=lse, x_mid=x_mid, h2=h2, m2=m2,
                                    r2=r2, pre=pre, u=u))
            x = x_out
        post, pm, pr = ops.norm_fwd(x, P[vp + "post_layernorm.weight"], P[vp + "post_layernorm.bias"], V.eps,
                                    save_stats=save)
        sv = None
        if save:
            sv = Saved(rows=rows, layers=layers, x_last=x, pm=pm, pr=pr, NI=NI)
        return x, post, sv

    def vision_backward(self, sv, dx, dpost=None):
        """dx: grad wrt x_last [NT, D] (bf16, consumed in place); dpost: grad wrt post-LN output."""
        V, P = self.cfg.vision, self.P
        vp = "vision_tower.vision_model."
        D = V.hidden
        NI = sv["NI"]
        NT = NI * V.n_patches
        gw = self.train_vision
        W = self.wlane
        if dpost is not None:
            ops.norm_bwd(sv["x_last"], P[vp + "post_layernorm.weight"], dpost, sv["pm"], sv["pr"], dx=dx,
                         dx_accum=True,
                         dweight=P.grad_view(vp + "post_layernorm.weight") if gw else None,
                         dbias=P.grad_view(vp + "post_layernorm.bias") if gw else None)
        for i in reversed(range(V.layers)):
            p = f"{vp}encoder.layers.{i}."
            s = sv["layers"][i]
            W2 = P[p + "mlp.fc2.weight"]
            du = ops.gemm(dx, W2.t())
            ev = None
            if gw:
                ev = W.run(lambda: (ops.gemm(dx.t(), s["u"].t(), out=P.grad_view(p + "mlp.fc2.weight"), accumulate=True),
                                    ops.colsum(dx, P.grad_view(p + "mlp.fc2.bias"))), dx, s["u"])
            dpre = ops.act_bwd(s["pre"], du, "gelu_tanh", out=du)
            dh2 = ops.gemm(dpre, P[p + "mlp.fc1.weight"].t())
            if gw:
                W.run(lambda: (ops.gemm(dpre.t(), s["h2"].t(), out=P.grad_view(p + "mlp.fc1.weight"), accumulate=True),
                               ops.colsum(dpre, P.grad_view(p + "mlp.fc1.bias"))), dpre, s["h2"])
            del du, dpre
            _wait(ev)   # dx is updated in place next
            ops.norm_bwd(s["x_mid"], P[p + "layer_norm2.weight"], dh2, s["m2"], s["r2"], dx=dx, dx_accum=True,
                         dweight=P.grad_view(p + "layer_norm2.weight") if gw else None,
                         dbias=P.grad_view(p + "layer_norm2.bias") if gw else None)
            do = ops.gemm(dx, P[p + "self_attn.out_proj.weight"].t())
            if gw:
                ev = W.run(lambda: (ops.gemm(dx.t(), s["o"].t(), out=P.grad_view(p + "self_attn.out_proj.weight"),
                                             accumulate=True),
                                    ops.colsum(dx, P.grad_view(p + "self_attn.out_proj.bias"))), dx, s["o"])
            dq, dk, dv = ops.attn_bwd(s["q"], s["k"], s["v"], s["o"], do, s["lse"], V.hd, causal=False)
            dqkv = ops.qkv_merge(dq, dk, dv, NI, V.n_patches, V.heads, V.heads, V.hd, V.hdp)
            del dq, dk, dv, do
            Wqkv = P.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight", 3 * D, D)
            dh = ops.gemm(dqkv, Wqkv.t())
            if gw:
                W.run(lambda: (ops.gemm(dqkv.t(), s["h"].t(), out=P.grad_span(p + "self_attn.q_proj.weight",
                                                                               p + "self_attn.v_proj.weight", 3 * D, D),
                                        accumulate=True),
                               ops.colsum(dqkv, P.grad_span(p + "self_attn.q_proj.bias", p + "self_attn.v_proj.bias", 1,
                                                            3 * D).view(-1))), dqkv, s["h"])
            del dqkv
            _wait(ev)
            ops.norm_bwd(s["x"], P[p + "layer_norm1.weight"], dh, s["m1"], s["r1"], dx=dx, dx_accum=True,
                         dweight=P.grad_view(p + "layer_norm1.weight") if gw else None,
                         dbias=P.grad_view(p + "layer_norm1.bias") if gw else None)
            sv["layers"][i] = None   # free activations as we go
        if gw:
            W.run(lambda: (ops.gemm(dx.t(), sv["rows"].t(), out=P.grad_view(vp + "embeddings.patch_embedding.weight"),
                                    accumulate=True),
                           ops.colsum(dx, P.grad_view(vp + "embeddings.patch_embedding.bias")),
                           ops.colsum(dx.view(NI, V.n_patches * D),
                                      P.grad_view(vp + "embeddings.position_embedding.weight").view(-1))),
                  dx, sv["rows"])

    # =========================================================== projector ====
    def projector_forward(self, x_last, save: bool):
        P = self.P
        pre = torch.empty((x_last.shape[0], self.cfg.text.hidden), dtype=torch.bfloat16,
                          device=self.device) if save else None
        z = ops.gemm(x_last, P["multi_modal_projector.linear_1.weight"], bias=P["multi_modal_projector.linear_1.bias"],
                     act=self.cfg.projector_act, aux=pre)
        feats = ops.gemm(z, P["multi_modal_projector.linear_2.weight"], bias=P["multi_modal_projector.linear_2.bias"])
        return feats, (Saved(x_last=x_last, pre=pre, z=z) if save else None)

    def projector_backward(self, s, dfeats, need_dx: bool):
        P = self.P
        gw = self.train_projector
        W = self.wlane
        dz = ops.gemm(dfeats, P["multi_modal_projector.linear_2.weight"].t())
        if gw:
            W.run(lambda: (ops.gemm(dfeats.t(), s["z"].t(), out=P.grad_view("multi_modal_projector.linear_2.weight"),
                                    accumulate=True),
                           ops.colsum(dfeats, P.grad_view("multi_modal_projector.linear_2.bias"))), dfeats, s["z"])
        dpre = ops.act_bwd(s["pre"], dz, self.cfg.projector_act, out=dz)
        if gw:
            W.run(lambda: (ops.gemm(dpre.t(), s["x_last"].t(), out=P.grad_view("multi_modal_projector.linear_1.weight"),
                                    accumulate=True),
                           ops.colsum(dpre, P.grad_view("multi_modal_projector.linear_1.bias"))), dpre, s["x_last"])
        if need_dx:
            return ops.gemm(dpre, P["multi_modal_projector.linear_1.weight"].t())
        return None

    # ============================================================ language ====
    def lm_forward(self, embeds, B, L, save: bool, kv_out: list | None = None):
        T, P = self.cfg.text, self.P
        M = B * L
        cos, sin = self._rope_for(L)
        lp = "language_model.model."
        qd, kd = T.heads * T.head_dim, T.kv_heads * T.head_dim
        x = embeds
        layers = []
        for i in range(T.layers):
            p = f"{lp}layers.{i}."
            Wqkv = P.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight", qd + 2 * kd, T.hidden)
            bqkv = P.span(p + "self_attn.q_proj.bias", p + "self_attn.v_proj.bias", 1, qd + 2 * kd).view(-1)
            h, _, r1 = ops.norm_fwd(x, P[p + "input_layernorm.weight"], None, T.eps, rms=True, save_stats=save)
            qkv = ops.gemm(h, Wqkv, bias=bqkv)
            q, k, v = ops.qkv_split(qkv, B, L, T.heads, T.kv_heads, T.head_dim, T.head_dim, cos, sin)
            del qkv
            if kv_out is not None:   # generate(): the prefill's roped keys / values seed the KV cache
                kv_out.append((k, v))
            o, lse = ops.attn_fwd(q, k, v, T.head_dim, causal=True, want_lse=save)
            o2 = o.view(M, qd)
            x_mid = ops.gemm(o2, P[p + "self_attn.o_proj.weight"], residual=x)
            h2, _, r2 = ops.norm_fwd(x_mid, P[p + "post_attention_layernorm.weight"], None, T.eps, rms=True,
                                     save_stats=save)
            Wgu = P.span(p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight", 2 * T.inter, T.hidden)
            if T.inter % 128 == 0:   # SwiGLU fused into the gate|up GEMM; gate|up kept only for the backward
                gu = torch.empty((M, 2 * T.inter), dtype=torch.bfloat16, device=self.device) if save else None
                a = ops.gemm(h2, Wgu, act="swiglu", aux=gu)
            else:
                gu = ops.gemm(h2, Wgu)
                a = ops.swiglu_fwd(gu, T.inter)
            x_out = ops.gemm(a, P[p + "mlp.down_proj.weight"], residual=x_mid)
            if save:
                layers.append(Saved(x=x, h=h, r1=r1, q=q, k=k, v=v, o=o2, lse=lse, x_mid=x_mid, h2=h2, r2=r2, gu=gu, a=a))
            else:
                del gu, a
            x = x_out
        hn, _, rf = ops.norm_fwd(x, P[lp + "norm.weight"], None, T.eps, rms=True, save_stats=save)
        sv = Saved(layers=layers, x_last=x, hn=hn, rf=rf, B=B, L=L) if save else None
        return hn, sv

    def lm_head_weight(self):
        T = self.cfg.text
        return self.P["language_model.model.embed_tokens.weight" if T.tie else "language_model.lm_head.weight"]

    def lm_head_grad(self):
        T = self.cfg.text
        return self.P.grad_view("language_model.model.embed_tokens.weight" if T.tie else "language_model.lm_head.weight")

    def logits(self, hn):
        return ops.gemm(hn, self.lm_head_weight())

    def lm_backward(self, sv, dhn, gscale=None, on_layer_done=None):
        """dhn: grad wrt the final-norm output [M, H] -> grad wrt inputs_embeds [M, H]."""
        T, P = self.cfg.text, self.P
        lp = "language_model.model."
        B, L = sv["B"], sv["L"]
        cos, sin = self._rope_for(L)
        qd, kd = T.heads * T.head_dim, T.kv_heads * T.head_dim
        gw = self.train_language
        W = self.wlane
        dx = ops.norm_bwd(sv["x_last"], P[lp + "norm.weight"], dhn, None, sv["rf"], rms=True,
                          dweight=P.grad_view(lp + "norm.weight") if gw else None)
        for i in reversed(range(T.layers)):
            p = f"{lp}layers.{i}."
            s = sv["layers"][i]
            da = ops.gemm(dx, P[p + "mlp.down_proj.weight"].t())
            ev = None
            if gw:
                ev = W.run(lambda: ops.gemm(dx.t(), s["a"].t(), out=P.grad_view(p + "mlp.down_proj.weight"),
                                            accumulate=True), dx, s["a"])
            dgu = ops.swiglu_bwd(s["gu"], da, T.inter)
            del da
            Wgu = P.span(p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight", 2 * T.inter, T.hidden)
            dh2 = ops.gemm(dgu, Wgu.t())
            if gw:
                W.run(lambda: ops.gemm(dgu.t(), s["h2"].t(), out=P.grad_span(p + "mlp.gate_proj.weight",
                                                                              p + "mlp.up_proj.weight",
                                                                              2 * T.inter, T.hidden),
                                       accumulate=True), dgu, s["h2"])
            del dgu
            _wait(ev)   # dx is updated in place next
            ops.norm_bwd(s["x_mid"], P[p + "post_attention_layernorm.weight"], dh2, None, s["r2"], dx=dx,
                         dx_accum=True, rms=True,
                         dweight=P.grad_view(p + "post_attention_layernorm.weight") if gw else None)
            do = ops.gemm(dx, P[p + "self_attn.o_proj.weight"].t())
            if gw:
                ev = W.run(lambda: ops.gemm(dx.t(), s["o"].t(), out=P.grad_view(p + "self_attn.o_proj.weight"),
                                            accumulate=True), dx, s["o"])
            dq, dk, dv = ops.attn_bwd(s["q"], s["k"], s["v"], s["o"], do, s["lse"], T.head_dim, causal=True)
            dqkv = ops.qkv_merge(dq, dk, dv, B, L, T.heads, T.kv_heads, T.head_dim, T.head_dim, cos, sin)
            del dq, dk, dv, do
            Wqkv = P.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight", qd + 2 * kd, T.hidden)
            dh = ops.gemm(dqkv, Wqkv.t())
            if gw:
                W.run(lambda: (ops.gemm(dqkv.t(), s["h"].t(), out=P.grad_span(p + "self_attn.q_proj.weight",
                                                                               p + "self_attn.v_proj.weight",
                                                                               qd + 2 * kd, T.hidden),
                                        accumulate=True),
                               ops.colsum(dqkv, P.grad_span(p + "self_attn.q_proj.bias", p + "self_attn.v_proj.bias", 1,
                                                            qd + 2 * kd).view(-1))), dqkv, s["h"])
            del dqkv
            _wait(ev)
            ops.norm_bwd(s["x"], P[p + "input_layernorm.weight"], dh, None, s["r1"], dx=dx, dx_accum=True, rms=True,
                         dweight=P.grad_view(p + "input_layernorm.weight") if gw else None)
            sv["layers"][i] = None
            if on_layer_done is not None:
                on_layer_done(i)
        return dx

    # ========================================================= full model ====
    def forward(self, input_ids, pixel_values, image_sizes, save: bool = False, want_post_ln: bool = False,
                kv_out: list | None = None):
        """LlavaOnevisionForConditionalGeneration.forward up to the final norm.

        input_ids [B, L] int64 (device), pixel_values [B, P, 3, 384, 384], image_sizes
        [B, 2] (host-readable).  Returns a dict with `hn` (final-norm hidden [B*L, H]),
        `post_ln` (vision post_layernorm output, the reference's hook, DT:110-121) and the
        saves for backward."""
        B, L = input_ids.shape
        Pn = pixel_values.shape[1]
        px = pixel_values.reshape(B * Pn, *pixel_values.shape[2:])
        x_last, post, vsave = self.vision_forward(px, save=save)
        feats, psave = self.projector_forward(x_last, save=save)
        src = self._src_map(input_ids, image_sizes.tolist() if hasattr(image_sizes, "tolist") else image_sizes, Pn)
        emb = ops.embed_assemble(input_ids.reshape(-1), src, self.P["language_model.model.embed_tokens.weight"], feats,
                                 self.P["image_newline"], self.err)
        del feats
        hn, lsave = self.lm_forward(emb, B, L, save=save, kv_out=kv_out)
        out = dict(hn=hn, src=src, ids=input_ids.reshape(-1))
        if want_post_ln:
            out["post_ln"] = post
        if save:
            out.update(vsave=vsave, psave=psave, lsave=lsave)
        return out

    def backward(self, fwd, dhn, dpost=None, gscale=None, on_layer_done=None):
        """Backward from d(final-norm hidden) and d(post-LN hook output) to every trainable grad."""
        T = self.cfg.text
        demb = self.lm_backward(fwd["lsave"], dhn, gscale, on_layer_done)
        _wait(self.tied_grad_event)   # the tied lm_head wgrad accumulates into the embedding grad too
        self.tied_grad_event = None
        NT = fwd["vsave"]["x_last"].shape[0] if fwd.get("vsave") else 0
        dfeats = torch.empty((NT, T.hidden), dtype=torch.bfloat16, device=self.device)
        ops.embed_bwd(fwd["ids"], fwd["src"], demb,
                      dtable=self.P.grad_view("language_model.model.embed_tokens.weight") if self.train_language else None,
                      dfeats=dfeats,
                      dnewline=self.P.grad_view("image_newline") if self.train_projector else None)
        del demb
        need_vision = self.train_vision
        dx_last = self.projector_backward(fwd["psave"], dfeats, need_dx=need_vision)
        if need_vision:
            self.vision_backward(fwd["vsave"], dx_last, dpost)
        if self.wlane is not None:
            self.wlane.join()
