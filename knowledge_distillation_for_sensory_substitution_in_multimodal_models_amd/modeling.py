"""LLaVA-OneVision (SigLIP + projector + anyres pack + Qwen2 + lm_head) on the HIP kernels.

The reference loads `LlavaOnevisionForConditionalGeneration` from transformers (DT:33-48)
and calls it as `model(input_ids=, pixel_values=, labels=, image_sizes=)` (DT:228, :238).
This module is the Python face of the library's model runtime (include/kdstep.h
kd_model_*: the forward and backward layer loops run in C++, csrc/model.hip, issuing the
kernels straight onto the caller's streams).  PyTorch allocates the parameters, the
workspaces and the outputs; every FLOP runs in libkdstep.so.

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

import ctypes as C
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as NV
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


def real_width_config(teacher: bool = False, layers: int = 2) -> LlavaConfig:
    """The REAL architectures (SigLIP 1152/4304, 16 x hd 72; Qwen2-7B 3584/18944, 28q/4kv
    hd 128; Qwen2-0.5B 896/4864, 14q/2kv hd 64; real vocabularies) cut to `layers` layers
    per tower: model-level parity at the real kernel shapes (tests/golden/model_real_*.npz)."""
    from dataclasses import replace
    base = TEACHER_7B if teacher else STUDENT_05B
    return replace(base, vision=replace(base.vision, layers=layers), text=replace(base.text, layers=layers))


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
        # called before the flat gradient is handed out: the owner of a backward that runs
        # on its own stream makes the reader's stream wait for it (kd_module)
        self.grad_fence = None
        if trainable:
            self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            self._grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            self.exp_avg = torch.zeros_like(self.master)
            self.exp_avg_sq = torch.zeros_like(self.master)
        self._views = {s.name: self.view(s.name) for s in self.specs}
        # region boundaries of the freeze masks (DT:468-523)
        first_proj = self.offsets["multi_modal_projector.linear_1.weight"][0]
        first_lm = self.offsets["language_model.model.embed_tokens.weight"][0]
        self.regions = {"vision": (0, first_proj), "projector": (first_proj, first_lm),
                        "language": (first_lm, self.numel)}

    @property
    def grad(self):
        """The flat fp32 gradient, complete on the current stream."""
        if self.grad_fence is not None:
            self.grad_fence()
        return self._grad

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


# ------------------------------------------------------- hub key layouts ----
def hub_key_to_445(k: str) -> str:
    """A LlavaOnevisionForConditionalGeneration state_dict key in either transformers layout
    -> the transformers-4.45 name the reference's checkpoints and this build use.

    4.45 (the reference's pin, and the hub's llava-onevision-qwen2-*-ov-hf safetensors):
    `vision_tower.vision_model.*`, `multi_modal_projector.*`, `image_newline`,
    `language_model.model.*`, `language_model.lm_head.weight` -- returned unchanged.
    5.x (installed here): `model.vision_tower.*`, `model.multi_modal_projector.*`,
    `model.image_newline`, `model.language_model.*`, `lm_head.weight`."""
    if k.startswith("model.vision_tower.vision_model."):      # 4.5x intermediate layout
        return "vision_tower.vision_model." + k[len("model.vision_tower.vision_model."):]
    if k.startswith("model.vision_tower."):
        return "vision_tower.vision_model." + k[len("model.vision_tower."):]
    if k.startswith("model.multi_modal_projector."):
        return k[len("model."):]
    if k == "model.image_newline":
        return "image_newline"
    if k.startswith("model.language_model.model."):
        return "language_model.model." + k[len("model.language_model.model."):]
    if k.startswith("model.language_model."):
        return "language_model.model." + k[len("model.language_model."):]
    if k == "lm_head.weight":
        return "language_model.lm_head.weight"
    return k


def hf_state_dict_to_445(sd: dict) -> dict:
    """Rename a whole state_dict (either layout) to the 4.45 names (hub_key_to_445)."""
    out = {}
    for k, v in sd.items():
        k4 = hub_key_to_445(k)
        if k4 in out:
            raise KeyError(f"{k} and another key both map to {k4}")
        out[k4] = v
    return out


# ------------------------------------------------------------------ helpers ----
def rope_tables(seq: int, hd: int, theta: float, device):
    """cos/sin [seq, hd/2] fp32 as HF's Qwen2RotaryEmbedding (inv_freq in fp32)."""
    inv = (1.0 / (theta ** (np.arange(0, hd, 2, dtype=np.int64).astype(np.float32) / hd))).astype(np.float32)
    f = np.arange(seq, dtype=np.float32)[:, None] * inv[None, :]
    return (torch.from_numpy(np.cos(f).astype(np.float32)).to(device),
            torch.from_numpy(np.sin(f).astype(np.float32)).to(device))


# priority of the training step's streams (lower = higher; 0 = default)
STREAM_PRIORITY_HIGH = -1   # the student chain's stream priority (DESIGN §3 Streams: measured best)


class WgradLane:
    """The weight-gradient stream of a trainable model: the runtime's backward issues every
    dW GEMM and bias column sum on it, beside the dgrad chain on the current stream
    (csrc/model.hip); `run` puts extra work there (the lm_head wgrad, kd_module), ordered
    after everything queued on the current stream, keeps its operands alive for it and
    returns an event; `join` makes the current stream wait for all of it."""

    def __init__(self, device):
        self.stream = torch.cuda.Stream(device=device, priority=STREAM_PRIORITY_HIGH)
        self.serial = False   # True: the weight gradients run on the current stream (measurement)

    def lane_stream(self):
        return torch.cuda.current_stream() if self.serial else self.stream

    def run(self, fn, *keep):
        if self.serial:
            fn()
            return None
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            fn()
        for t in keep:
            if t is not None:
                t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    def join(self):
        if not self.serial:
            torch.cuda.current_stream().wait_stream(self.stream)


def native_config(cfg: LlavaConfig) -> NV.KdModelConfig:
    V, T = cfg.vision, cfg.text
    return NV.KdModelConfig(V.hidden, V.inter, V.layers, V.heads, V.patch, V.image, V.eps,
                            T.hidden, T.inter, T.layers, T.heads, T.kv_heads, T.head_dim, T.vocab, int(T.tie),
                            T.rope_theta, T.eps, cfg.image_token_id, ops.ACTS[cfg.projector_act])


def native_layout(cfg: LlavaConfig) -> list[tuple[str, int, int]]:
    """(name, offset, numel) of every parameter as the library lays out the flat buffer."""
    c = native_config(cfg)
    lib = NV.lib()
    out = []
    name = C.create_string_buffer(256)
    off, n, r, k = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
    for i in range(lib.kd_model_param_count(C.byref(c))):
        NV.call("kd_model_param_info", C.byref(c), i, name, 256, C.byref(off), C.byref(n), C.byref(r), C.byref(k))
        out.append((name.value.decode(), off.value, n.value))
    return out


# --------------------------------------------------------------------- model ----
# fp8 (e4m3) teacher policies: which linear families run on the fp8 GEMM (kd_fp8_family bits)
FP8_FAMILIES = {
    "all": NV.KD_FP8_ALL,
    "lm": NV.KD_FP8_LM_ATTN | NV.KD_FP8_LM_MLP | NV.KD_FP8_LM_HEAD,
    "lm_body": NV.KD_FP8_LM_ATTN | NV.KD_FP8_LM_MLP,
    "lm_mlp": NV.KD_FP8_LM_MLP,
    "none": 0,
}


class LlavaOnevisionModel:
    """One LLaVA-OneVision instance (teacher or student) on a ParamStore, driven through the
    library's model runtime (one forward call, one backward call per step)."""

    def __init__(self, cfg: LlavaConfig, device, trainable: bool = False, seed: int | None = None,
                 cpu_rng: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        self.P = ParamStore(cfg, device, trainable)
        if seed is not None:
            self.P.init_(seed, cpu_rng=cpu_rng)
        self._rope = {}
        self._maps = {}
        self._ws = {}
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        # which regions receive weight gradients (freeze masks, DT:468-523)
        self._train = [trainable] * 3   # vision, projector, language
        self.wlane = WgradLane(self.device) if (trainable and self.device.type == "cuda") else None
        self._ncfg = native_config(cfg)
        if NV.lib().kd_model_param_numel(C.byref(self._ncfg)) != self.P.numel:
            raise RuntimeError("flat parameter layout differs from the library's (kd_model_param_info)")
        h = C.c_void_p()
        NV.call("kd_model_create", C.byref(self._ncfg), self.P.flat.data_ptr(),
                self.P.grad.data_ptr() if trainable else None, C.byref(h))
        self._h = h
        self.fp8 = False
        # fp32 residual streams (kd_model_set_residual_f32), as the reference's fp32 / autocast
        # step keeps them: the student both towers; the teacher its SigLIP tower (cheap: 1152
        # wide; its pooled post-LN features feed NT-Xent) but not its 3584-wide Qwen2 stream.
        # With bf16 streams the tiny fixtures' pooled ViT features sat 1.7-2.0 % from the fp32
        # reference, with fp32 streams 0.15-0.17 % (tools/vit_feature_check.py), and the student
        # rounding after every residual add moved the gradient norm by +0.12 % (tools/grad_bias_study.py)
        self.residual_f32 = (False, False)
        self.fp8_families = 0
        self.lm_stream_f32 = False
        self.set_residual_f32(*self._default_streams())

    def set_residual_f32(self, vision: bool, language: bool):
        """fp32 residual streams of the SigLIP / Qwen2 towers (kd_model_set_residual_f32)."""
        NV.call("kd_model_set_residual_f32", self._h, int(vision), int(language))
        self.residual_f32 = (bool(vision), bool(language))
        self._ws = {}   # the workspaces' stream buffers change size

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is None or not h.value:
            return
        try:
            NV.lib().kd_model_destroy(h)
        except Exception:   # interpreter shutdown: the module's globals are already torn down
            return
        self._h = None

    # -- freeze masks mirroring DT:468-523 (applied to the student), kept in the runtime too
    def set_trainable(self, vision: bool, projector: bool, language: bool):
        self._train = [bool(vision), bool(projector), bool(language)]
        NV.call("kd_model_set_trainable", self._h, *map(int, self._train))

    def _flag(i):
        def get(self):
            return self._train[i]

        def put(self, v):
            t = list(self._train)
            t[i] = bool(v)
            self.set_trainable(*t)
        return property(get, put)

    train_vision, train_projector, train_language = _flag(0), _flag(1), _flag(2)
    del _flag

    def _rope_for(self, L):
        if L not in self._rope:
            self._rope[L] = rope_tables(L, self.cfg.text.head_dim, self.cfg.text.rope_theta, self.device)
        return self._rope[L]

    def _src_map(self, input_ids, image_sizes, tiles=0):
        """Per-token source rows of inputs_embeds: the anyres pack plan (kd_anyres_batch_map,
        host, cached per image_sizes; tiles = 0: feature rows over the compact real tiles)
        expanded on the device by kd_image_src_map."""
        key = (tuple(tuple(int(v) for v in hw) for hw in image_sizes), tiles)
        if key not in self._maps:
            B = len(key[0])
            isz = np.asarray(key[0], dtype=np.int64).reshape(B, 2)
            ld = max(anyres.num_image_tokens(hw) for hw in key[0])
            arr = np.empty((B, ld), dtype=np.int32)
            lens = np.empty(B, dtype=np.int32)
            NV.call("kd_anyres_batch_map", isz.ctypes.data, B, tiles, arr.ctypes.data, ld, lens.ctypes.data)
            self._maps[key] = (torch.from_numpy(arr).to(self.device), torch.from_numpy(lens).to(self.device))
        maps, lens = self._maps[key]
        return ops.image_src_map(input_ids, self.cfg.image_token_id, maps, lens, self.err)

    # -- weights from a hub / transformers state_dict
    def load_hf_state_dict(self, sd: dict, strict: bool = True):
        """Load `LlavaOnevisionForConditionalGeneration.state_dict()` weights in the
        transformers-4.45 or 5.x key layout (hub_key_to_445) into the flat buffer (bf16; the
        fp32 master of a trainable model too); a frozen fp8 model is re-quantised."""
        seen = self.P.load_state_dict(hf_state_dict_to_445(sd), strict=strict)
        if self.fp8:
            self.enable_fp8(self.fp8_families)
        return seen

    # -- fp8 teacher (BASELINE config c4)
    def enable_fp8(self, families="all"):
        """Quantise every linear weight to e4m3 with per-output-channel scales (kd_model_quantize_fp8,
        on the current stream) and run the forward's linears of `families` (FP8_FAMILIES name or
        kd_fp8_family bits) on the fp8 GEMM from now on (per-token activation scales); the other
        linears keep the bf16 GEMM.  Frozen models only; re-run after the weights change."""
        if self.P.trainable:
            raise RuntimeError("fp8 weights are for the frozen teacher (no grad buffer)")
        fam = FP8_FAMILIES[families] if isinstance(families, str) else int(families)
        NV.call("kd_model_set_fp8", self._h, None, None)   # unbind while the policy changes
        # the fp8 GEMM adds a bf16 residual only: a tower whose residual linears go fp8 keeps a
        # bf16 stream (the defaults otherwise: _default_streams)
        v, t = self._default_streams()
        self.set_residual_f32(v and not fam & NV.KD_FP8_VISION,
                              t and not fam & (NV.KD_FP8_LM_ATTN | NV.KD_FP8_LM_MLP))
        NV.call("kd_model_set_fp8_families", self._h, fam)
        self.fp8_families = fam
        lib = NV.lib()
        n = lib.kd_model_fp8_scale_count(self._h)
        self._f8q = torch.empty(self.P.numel, dtype=torch.uint8, device=self.device)
        self._f8s = torch.empty(max(n, 1), dtype=torch.float32, device=self.device)
        NV.call("kd_model_quantize_fp8", self._h, self._f8q.data_ptr(), self._f8s.data_ptr(), ops._stream())
        NV.call("kd_model_set_fp8", self._h, self._f8q.data_ptr(), self._f8s.data_ptr())
        self._ws = {}   # the forward workspace gains the activation-quantisation buffers
        self.fp8 = True

    def disable_fp8(self):
        NV.call("kd_model_set_fp8", self._h, None, None)
        self._f8q = self._f8s = None
        self.set_residual_f32(*self._default_streams())
        self._ws = {}
        self.fp8 = False

    def _default_streams(self):
        """(vision, language) fp32 residual streams: both for the trainable student, the
        SigLIP tower only for a frozen teacher unless `lm_stream_f32` is set (its 3584-wide
        Qwen2 stream in fp32 too: the c1 reference teacher's precision, LB:29-33)."""
        return True, bool(self.P.trainable) or self.lm_stream_f32

    def set_lm_stream_f32(self, on: bool):
        """Default precision of the Qwen2 residual stream of a frozen model (the teacher):
        fp32 (on) or bf16.  The fp8 path keeps bf16 where its residual linears run fp8."""
        self.lm_stream_f32 = bool(on)
        if self.fp8:
            self.enable_fp8(self.fp8_families)
        else:
            self.set_residual_f32(*self._default_streams())

    def _workspace(self, key, nbytes):
        """One cached workspace per call shape: a save=1 forward's workspace holds the
        activations its backward reads, so it is only rewritten by the next forward."""
        ws = self._ws.get(key)
        if ws is None or ws.numel() < nbytes:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws

    def lm_head_weight(self):
        T = self.cfg.text
        return self.P["language_model.model.embed_tokens.weight" if T.tie else "language_model.lm_head.weight"]

    def lm_head_grad(self):
        T = self.cfg.text
        return self.P.grad_view("language_model.model.embed_tokens.weight" if T.tie else "language_model.lm_head.weight")

    def logits(self, hn):
        return ops.gemm(hn, self.lm_head_weight())

    # ========================================================= full model ====
    def forward(self, input_ids, pixel_values, image_sizes, save: bool = False, want_post_ln: bool = False,
                kv_out: list | None = None, want_logits: bool = False, row_stats: tuple | None = None):
        """LlavaOnevisionForConditionalGeneration.forward (kd_model_forward).

        input_ids [B, L] int64 (device), pixel_values [B, P, 3, 384, 384] (bf16 / fp32),
        image_sizes [B, 2] (host-readable).  Returns a dict with `hn` (final-norm hidden
        [B*L, H]), `post_ln` (vision post_layernorm output, the reference's hook, DT:110-121),
        `logits` [B*L, V] (want_logits), `tile_counts` (each sample's real vision tiles, the
        post_ln row groups) and, with save, the workspace the backward reads.
        kv_out (a list) receives each layer's roped (k, v) [B, kv_heads, L, head_dim].
        row_stats = (vs, inv_t, top2) with want_logits: `row_stats` [B*L, ceil(V/256), 8] fp32, the
        lm_head epilogue's per-row softmax statistics for the KD loss (kd_model_set_row_stats)."""
        T, V = self.cfg.text, self.cfg.vision
        B, L = input_ids.shape
        P = pixel_values.shape[1]
        sizes = image_sizes.tolist() if hasattr(image_sizes, "tolist") else image_sizes
        # the vision tower runs each image's REAL tiles only (base + anyres grid; HF drops the
        # zero tiles _pad_for_batching added: pix_val[:num_patch]), so a mixed batch
        # (336x336: 2 tiles, 480x640: 5) hooks exactly the reference's tile features
        counts = [anyres.num_tiles(tuple(int(v) for v in hw)) for hw in sizes]
        if any(n > P for n in counts):
            raise RuntimeError(f"pixel_values has {P} tiles per sample; image_sizes need {max(counts)}")
        px = pixel_values.reshape(B * P, *pixel_values.shape[2:])
        if any(n != P for n in counts):
            # the compact-tile index, cached per (tile counts, P) like the anyres maps: no
            # pageable host-to-device copy on every forward of a mixed batch
            key = ("tiles", tuple(counts), P)
            idx = self._maps.get(key)
            if idx is None:
                idx = torch.tensor([b * P + t for b in range(B) for t in range(counts[b])], device=px.device)
                self._maps[key] = idx
            px = px.index_select(0, idx)
        px = px.contiguous()
        tiles = int(sum(counts))   # vision tiles of the batch
        if px.dtype not in (torch.bfloat16, torch.float32):
            raise RuntimeError(f"pixel_values: bf16 or fp32, got {px.dtype}")
        ids = input_ids.contiguous()
        src = self._src_map(ids, sizes, 0)
        cos, sin = self._rope_for(L)
        lib = NV.lib()
        nb = lib.kd_model_forward_workspace_size(self._h, B, L, tiles, int(save))
        ws = self._workspace(("fwd", B, L, tiles, bool(save)), nb)
        dev = self.device
        hn = torch.empty((B * L, T.hidden), dtype=torch.bfloat16, device=dev)
        post = torch.empty((tiles * V.n_patches, V.hidden), dtype=torch.bfloat16, device=dev) \
            if want_post_ln else None
        logits = torch.empty((B * L, T.vocab), dtype=torch.bfloat16, device=dev) if want_logits else None
        kvk = kvv = None
        if kv_out is not None:
            ks = [torch.empty((B, T.kv_heads, L, T.head_dim), dtype=torch.bfloat16, device=dev) for _ in range(T.layers)]
            vs = [torch.empty_like(k) for k in ks]
            kv_out.extend(zip(ks, vs))
            kvk = (C.c_void_p * T.layers)(*[k.data_ptr() for k in ks])
            kvv = (C.c_void_p * T.layers)(*[v.data_ptr() for v in vs])
        rst = None
        if row_stats is not None and want_logits:
            vs, inv_t, top2 = row_stats
            rst = torch.empty((B * L, (T.vocab + 255) // 256, 8), dtype=torch.float32, device=dev)
            NV.call("kd_model_set_row_stats", self._h, rst.data_ptr(), int(vs), float(inv_t), int(bool(top2)))
        try:
            NV.call("kd_model_forward", self._h, ids.data_ptr(), px.data_ptr(), ops._DT[px.dtype], src.data_ptr(),
                    cos.data_ptr(), sin.data_ptr(), B, L, tiles, int(save), ws.data_ptr(), ws.numel(), hn.data_ptr(),
                    ops._ptr(post), ops._ptr(logits), kvk, kvv, self.err.data_ptr(), ops._stream())
        finally:
            if rst is not None:   # the handle never keeps a pointer past the call that owns it
                NV.call("kd_model_set_row_stats", self._h, None, 0, 1.0, 0)
        out = dict(hn=hn, src=src, ids=ids, shape=(B, L, tiles), tile_counts=counts)
        if rst is not None:
            out["row_stats"] = rst
        if want_post_ln:
            out["post_ln"] = post
        if want_logits:
            out["logits"] = logits
        if save:
            out["ws"] = ws
        return out

    def backward(self, fwd, dhn, dpost=None, on_layer_done=None):
        """Backward of a save=True forward from d(final-norm hidden) and d(post-LN hook
        output) into every trainable grad (kd_model_backward).  Weight gradients run on
        the wgrad lane; the current stream has joined it when this returns."""
        if "ws" not in fwd:
            raise RuntimeError("backward needs a forward run with save=True")
        B, L, tiles = fwd["shape"]
        if dpost is not None:
            # ABI 7: the gradient of each tile's MEAN post_ln feature, fp32 [tiles, v_hidden] (the
            # bf16 per-row gradient of ABI <= 6 would be read as the wrong type and shape)
            if dpost.dtype != torch.float32 or not dpost.is_contiguous() or \
                    tuple(dpost.shape) != (tiles, self.cfg.vision.hidden):
                raise RuntimeError(f"backward: dpost must be a contiguous fp32 [{tiles}, {self.cfg.vision.hidden}] "
                                   f"tile gradient, got {tuple(dpost.shape)} {dpost.dtype}")
        cos, sin = self._rope_for(L)
        nb = NV.lib().kd_model_backward_workspace_size(self._h, B, L, tiles)
        ws = self._workspace(("bwd", B, L, tiles), nb)
        cb = NV.LAYER_CB(lambda user, i: on_layer_done(i)) if on_layer_done is not None else NV.LAYER_CB()
        NV.call("kd_model_backward", self._h, fwd["ws"].data_ptr(), fwd["ids"].data_ptr(), fwd["src"].data_ptr(),
                cos.data_ptr(), sin.data_ptr(), B, L, tiles, dhn.contiguous().data_ptr(), ops._ptr(dpost),
                ws.data_ptr(), ws.numel(), ops._stream(), self.wlane.lane_stream().cuda_stream, cb, None)
