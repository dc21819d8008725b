"""Python-side launchers of the C-ABI kernels (device tensors in, device tensors out).

PyTorch is plumbing here: it allocates device memory and provides the stream; every
FLOP runs in libkdstep.so.  There is no CPU or torch fallback for any op.
"""
from __future__ import annotations

import contextlib
import ctypes as C

import torch

from . import _native as NV

_WS: dict = {}


class KernelTimer:
    """GEMM launch timing for bench.py's roofline pass: the library brackets every kd_gemm
    launch (ops.gemm and the model runtime's own) with HIP events on its launch stream
    while enabled (include/kdstep.h kd_timer_*)."""

    @property
    def enabled(self):
        return getattr(self, "_on", False)

    @enabled.setter
    def enabled(self, on):
        self._on = bool(on)
        NV.lib().kd_timer_enable(int(self._on))

    def reset(self):
        NV.lib().kd_timer_reset()

    def records(self):
        """[(key, flops, ms)], key = "<kind>:<M>x<N>x<K>:<out dtype>[:acc]" (synchronises)."""
        lib = NV.lib()
        key = C.create_string_buffer(128)
        fl, ms = C.c_double(), C.c_float()
        out = []
        for i in range(lib.kd_timer_count()):
            NV.call("kd_timer_read", i, key, 128, C.byref(fl), C.byref(ms))
            out.append((key.value.decode(), fl.value, ms.value))
        return out

    def summary(self, kind, where=None):
        """Totals of one kind; where(M, N, K) selects shapes (None: all)."""
        recs = [r for r in self.records() if r[0].split(":", 1)[0] == kind]
        if where is not None:
            recs = [r for r in recs if where(*map(int, r[0].split(":")[1].split("x")))]
        if not recs:
            return None
        ms = [r[2] for r in recs]
        flops = sum(r[1] for r in recs)
        return dict(launches=len(recs), total_ms=sum(ms), avg_ms=sum(ms) / len(ms), flops=flops,
                    flops_per_launch=flops / len(recs))

    def kinds(self):
        return sorted({r[0].split(":", 1)[0] for r in self.records()})

    def by_shape(self, top=25):
        """Per (layouts, M, N, K, out dtype) totals, heaviest first (tuning aid)."""
        agg = {}
        for key, fl, ms in self.records():
            t = agg.setdefault(key, [0, 0.0, fl])
            t[0] += 1
            t[1] += ms
        rows = sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]
        return [dict(shape=k, launches=n, total_ms=round(ms, 3), avg_us=round(1e3 * ms / n, 2),
                     tflops=round(fl * n / (ms * 1e-3) / 1e12, 1)) for k, (n, ms, fl) in rows]


TIMER = KernelTimer()

# fp32 split-K partial planes, one buffer per (stream, device); the library's cost model
# never plans more splits than fit
GEMM_SPLITK_WS = 384 << 20


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _workspace(key, nbytes: int, device) -> torch.Tensor:
    buf = _WS.get((key, device))
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=device)
        _WS[(key, device)] = buf
    return buf


def _require(t: torch.Tensor, dtype, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"{name}: expected a device tensor (no CPU path)")
    if t.dtype != dtype:
        raise RuntimeError(f"{name}: expected {dtype}, got {t.dtype}")


# ------------------------------------------------------------------ KD loss ----
def kd_loss_student_stats(student_logits: torch.Tensor, temperature: float = 1.0,
                          out: torch.Tensor | None = None) -> torch.Tensor:
    """The student half of the KD loss's per-row statistics (include/kdstep.h
    kd_loss_student_stats): fp32 [rows, 4] = {max, sum exp((s - max)/T), sum exp(s - max), 0}
    of every row of student_logits [..., V_s] (bf16, rows uniformly strided).  For
    kd_loss_fwd_bwd(s_stats=...) on the same rows and temperature."""
    _require(student_logits, torch.bfloat16, "student_logits")
    V_s = student_logits.shape[-1]
    x = student_logits.reshape(-1, V_s)
    if x.stride(1) != 1:
        raise RuntimeError("student_logits: contiguous last dim expected")
    rows = x.shape[0]
    o = out if out is not None else torch.empty((rows, 4), dtype=torch.float32, device=x.device)
    _require(o, torch.float32, "out")
    if not o.is_contiguous() or o.numel() != rows * 4:
        raise RuntimeError("out: expected a contiguous [rows, 4] fp32 tensor")
    NV.call("kd_loss_student_stats", _ptr(x), x.stride(0), V_s, rows, float(temperature), _ptr(o), _stream())
    return o



VARIANTS = {"none": NV.KD_LOSS_NONE, "loca": NV.KD_LOSS_LOCA, "kl": NV.KD_LOSS_KL,
            "kl_logtarget": NV.KD_LOSS_KL_LOGTARGET}


def kd_loss_fwd_bwd(student_logits: torch.Tensor, teacher_logits: torch.Tensor | None,
                    labels: torch.Tensor, variant: str, temperature: float = 1.0, alpha: float = 0.8,
                    kd_weight: float = 1.0, ce_weight: float = 1.0, grad_scale: float = 1.0,
                    clamp_min: float = 1e-8, teacher_ce: bool = True, want_grad: bool = True,
                    check: bool = False, loss_out: torch.Tensor | None = None, out_scale: float = 1.0,
                    accumulate: bool = False, dlogits_out: torch.Tensor | None = None,
                    err_out: torch.Tensor | None = None, row_base: int = 0,
                    dscale: torch.Tensor | None = None, dscale_given: bool = False,
                    s_row_stats: torch.Tensor | None = None, t_row_stats: torch.Tensor | None = None,
                    s_stats: torch.Tensor | None = None, loca_path: str = "auto", rr_poll_us: int | None = None,
                    standin_count: torch.Tensor | None = None):
    """Fused KD-loss forward + backward (include/kdstep.h kd_loss_fwd_bwd).

    student_logits [B, L, V_s] bf16 (last dim contiguous), teacher_logits [B, L, V_t] bf16,
    labels [B, L] int64.  Returns (loss4, dlogits): loss4 = fp32 [4] =
    (kd_term, student_ce, teacher_ce, total); dlogits bf16 [B, L, V_s] or None.

    Loss groups: loss_out / out_scale / accumulate let consecutive calls on
    sub-batches average their terms on the device; dlogits_out receives the gradient rows
    of this call.  err_out (device int32[4], caller-zeroed) collects label-range errors
    without a host sync (kd_loss_params.err_out).  dscale (device fp32 [1]): the dlogits are
    stored relative to the scale written there (or read from there, dscale_given), which
    the consumer multiplies back in fp32 (kd_loss_params.dscale: the CE one-hot element
    stays exact in bf16).  s_row_stats / t_row_stats (fp32 [B*L, ceil(V / 256), 8], these rows):
    the lm_head GEMMs' row statistics (gemm(row_stats=...), modeling set_row_stats) in place of
    the loss's own pass over the logits (kd_loss_params.s_row_stats / t_row_stats).
    s_stats (fp32 [B*L, 4], these rows, same temperature): kd_loss_student_stats' output, so the
    loss reads only the teacher's logits for its statistics (kd_loss_params.s_stats; same bits).
    loca_path "auto" (the register-resident slices where they fit) or "two_read" (k_loss_grad_loca);
    rr_poll_us: the register-resident kernel's partner poll budget (None = 200 us; 0 = every partner
    partial recomputed by the waiting slice); standin_count (device int32 [1]) += the partials that
    were recomputed (kd_loss_params.loca_path / rr_poll_us_p1 / standin_count).
    """
    B, L, V_s = student_logits.shape
    _require(student_logits, torch.bfloat16, "student_logits")
    _require(labels, torch.int64, "labels")
    if student_logits.stride(2) != 1 or student_logits.stride(0) != L * student_logits.stride(1):
        raise RuntimeError("student_logits: rows must be uniformly strided with a contiguous last dim")
    labels = labels.contiguous()
    v = VARIANTS[variant]
    if teacher_logits is not None:
        _require(teacher_logits, torch.bfloat16, "teacher_logits")
        if teacher_logits.stride(2) != 1 or teacher_logits.stride(0) != L * teacher_logits.stride(1):
            raise RuntimeError("teacher_logits: rows must be uniformly strided")
        V_t, ld_t = teacher_logits.shape[2], teacher_logits.stride(1)
    else:
        if v != NV.KD_LOSS_NONE:
            raise RuntimeError(f"kd_loss variant {variant} needs teacher logits")
        V_t, ld_t = 0, 0
    dev = student_logits.device
    loss = loss_out if loss_out is not None else torch.empty(4, dtype=torch.float32, device=dev)
    if want_grad:
        dl = dlogits_out if dlogits_out is not None else torch.empty((B, L, V_s), dtype=torch.bfloat16, device=dev)
        if dl.shape[-1] != V_s or dl.stride(-1) != 1 or dl.numel() != B * L * V_s:
            raise RuntimeError("dlogits_out: expected a contiguous [B, L, V_s] view")
    else:
        dl = None
    if err_out is not None:
        _require(err_out, torch.int32, "err_out")
    if dscale is not None:
        _require(dscale, torch.float32, "dscale")
    for nm, t, V in (("s_row_stats", s_row_stats, V_s), ("t_row_stats", t_row_stats, V_t)):
        if t is not None:
            _require(t, torch.float32, nm)
            if not t.is_contiguous() or t.numel() != B * L * ((V + 255) // 256) * 8:
                raise RuntimeError(f"{nm}: expected a contiguous [B*L, ceil(V/256), 8] fp32 block of these rows")
    if (s_row_stats is None) != (t_row_stats is None) and teacher_logits is not None:
        raise RuntimeError("s_row_stats and t_row_stats: both or neither")
    if s_stats is not None:
        _require(s_stats, torch.float32, "s_stats")
        if not s_stats.is_contiguous() or s_stats.numel() != B * L * 4:
            raise RuntimeError("s_stats: expected a contiguous [B*L, 4] fp32 block of these rows (kd_loss_student_stats)")
    nbytes = NV.lib().kd_loss_workspace_size(B, L, V_s)
    ws = _workspace("kd_loss", nbytes, dev)
    prm = NV.KdLossParams(v, float(temperature), float(alpha), float(kd_weight), float(ce_weight),
                         float(grad_scale), float(clamp_min), 1 if teacher_ce else 0, float(out_scale),
                         1 if accumulate else 0, _ptr(err_out), int(row_base), _ptr(dscale),
                         1 if dscale_given else 0, _ptr(s_row_stats), _ptr(t_row_stats), _ptr(s_stats),
                         {"auto": 0, "two_read": 1}[loca_path], 0 if rr_poll_us is None else int(rr_poll_us) + 1,
                         _ptr(standin_count))
    if standin_count is not None:
        _require(standin_count, torch.int32, "standin_count")
    NV.call("kd_loss_fwd_bwd", _ptr(teacher_logits), ld_t, V_t, _ptr(student_logits),
           student_logits.stride(1), V_s, _ptr(labels), B, L, prm, _ptr(loss), _ptr(dl),
           V_s, _ptr(ws), ws.numel(), _stream())
    if check:
        NV.call("kd_loss_check", _ptr(ws), _stream())
    return loss, dl


# --------------------------------------------------------------------- GEMM ----
ACTS = {None: NV.KD_ACT_NONE, "none": NV.KD_ACT_NONE, "gelu_tanh": NV.KD_ACT_GELU_TANH,
        "gelu_erf": NV.KD_ACT_GELU_ERF, "silu": NV.KD_ACT_SILU, "swiglu": NV.KD_ACT_SWIGLU,
        "dgelu_tanh": NV.KD_ACT_DGELU_TANH, "dswiglu": NV.KD_ACT_DSWIGLU}
_DT = {torch.bfloat16: NV.KD_DTYPE_BF16, torch.float32: NV.KD_DTYPE_F32}


def _operand(x: torch.Tensor, name: str):
    """(ptr, ld, layout, rows, k) of a 2-D bf16 operand; MN-major if it is a transposed view."""
    _require(x, torch.bfloat16, name)
    if x.dim() != 2:
        raise RuntimeError(f"{name}: expected 2-D")
    r, k = x.shape
    if x.stride(1) == 1 and (x.stride(0) >= k or r == 1):
        return x.data_ptr(), max(x.stride(0), k), NV.KD_LAYOUT_K_MAJOR
    if x.stride(0) == 1 and (x.stride(1) >= r or k == 1):
        return x.data_ptr(), max(x.stride(1), r), NV.KD_LAYOUT_MN_MAJOR
    raise RuntimeError(f"{name}: needs a unit stride in one dimension")


def _gemm_desc(a, b, out, bias, act, residual, aux, alpha, alpha_dev, accumulate, out_dtype, residual_row_mod,
               variant, split_k):
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise RuntimeError(f"gemm: K mismatch {K} vs {K2}")
    pa, lda, la = _operand(a, "gemm.a")
    pb, ldb, lb = _operand(b, "gemm.b")
    if out is None:
        out = torch.empty((M, N // 2 if act == "swiglu" else (2 * N if act == "dswiglu" else N)), dtype=out_dtype,
                          device=a.device)
    if out.stride(1) != 1:
        raise RuntimeError("gemm: out must have a contiguous last dim")
    d = NV.KdGemmDesc()
    d.M, d.N, d.K, d.a_layout, d.b_layout = M, N, K, la, lb
    d.A, d.lda, d.B, d.ldb = pa, lda, pb, ldb
    d.C, d.ldc, d.c_dtype, d.accumulate = out.data_ptr(), out.stride(0), _DT[out.dtype], int(accumulate)
    d.alpha, d.alpha_dev = float(alpha), _ptr(alpha_dev)
    if bias is not None:
        d.bias, d.bias_dtype = bias.data_ptr(), _DT[bias.dtype]
    d.act = ACTS[act]
    d.variant = int(variant)
    d.split_k = int(split_k)
    if split_k != 1 or variant == 21:   # split-K partial planes / stream-K tickets + partial tiles
        ws = _workspace(("gemm_splitk", _stream()), GEMM_SPLITK_WS, a.device)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
    if residual is not None:
        if residual.dtype not in _DT or not residual.is_cuda:
            raise RuntimeError("gemm.residual: expected a bf16 or fp32 device tensor")
        d.residual, d.ldr = residual.data_ptr(), residual.stride(0)
        d.residual_row_mod = int(residual_row_mod)
        d.residual_dtype = _DT[residual.dtype]
    if aux is not None:
        _require(aux, torch.bfloat16, "gemm.aux")
        d.aux, d.ld_aux = aux.data_ptr(), aux.stride(0)
    return d, out, M, N, K, la, lb


def gemm_qkv(x: torch.Tensor, w: torch.Tensor, bias, q, k, v, S: int, nq: int, nkv: int, hd: int, hdp: int,
             cos=None, sin=None, variant: int = 0, b_pretiled: torch.Tensor | None = None):
    """Fused q|k|v projection: x [M, K] @ w[N, K]^T + bias written straight to head-major q
    [B, nq, S, hdp], k / v [B, nkv, S, hdp] (+ RoPE with cos / sin [S, hd/2] fp32), the
    padding zeroed (include/kdstep.h kd_qkv_scatter) — equal to gemm() + qkv_split()."""
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _require(t, torch.bfloat16, f"gemm_qkv.{n}")
        if not t.is_contiguous():
            raise RuntimeError(f"gemm_qkv.{n}: contiguous head-major tensor expected")
    sc = NV.KdQkvScatter(q.data_ptr(), k.data_ptr(), v.data_ptr(), _ptr(cos), _ptr(sin), int(S), int(nq), int(nkv),
                         int(hd), int(hdp))
    d, _, M, N, K, la, lb = _gemm_desc(x, w, q.view(-1, 1), bias, None, None, None, 1.0, None, False,
                                       torch.bfloat16, 0, variant, 1)
    d.C, d.ldc = None, 0
    d.qkv = C.cast(C.pointer(sc), C.c_void_p)
    if b_pretiled is not None:
        _set_pretiled(d, b_pretiled, N, K, False)
    NV.call("kd_gemm", C.byref(d), _stream())
    return q, k, v


def gemm_plan(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, *, bias=None, act=None,
              residual=None, aux=None, alpha: float = 1.0, alpha_dev=None, accumulate: bool = False,
              out_dtype=torch.bfloat16, residual_row_mod: int = 0, variant: int = 0, split_k: int = 0):
    """(kernel variant, K splits, unsplit leading tiles) that gemm() with these arguments runs
    (kd_gemm_plan; inspection only, nothing is launched)."""
    d = _gemm_desc(a, b, out, bias, act, residual, aux, alpha, alpha_dev, accumulate, out_dtype, residual_row_mod,
                   variant, split_k)[0]
    v, s_, dp = C.c_int32(), C.c_int32(), C.c_int32()
    NV.call("kd_gemm_plan", C.byref(d), C.byref(v), C.byref(s_), C.byref(dp))
    return v.value, s_.value, dp.value


_SPLIT_DEFAULT = [0]


@contextlib.contextmanager
def gemm_split_default(split_k: int):
    """Within the block, gemm(split_k=0) calls use `split_k` instead (0 = cost model)."""
    prev = _SPLIT_DEFAULT[0]
    _SPLIT_DEFAULT[0] = int(split_k)
    try:
        yield
    finally:
        _SPLIT_DEFAULT[0] = prev


def gemm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, *, bias=None, act=None,
         residual=None, aux=None, alpha: float = 1.0, alpha_dev=None, accumulate: bool = False,
         out_dtype=torch.bfloat16, residual_row_mod: int = 0, variant: int = 0, split_k: int = 0,
         row_stats: torch.Tensor | None = None, row_stats_vs: int = 0, row_stats_inv_t: float = 1.0,
         row_stats_top2: bool = False, b_pretiled: torch.Tensor | None = None) -> torch.Tensor:
    """out[M, N] = epilogue(alpha * a[M, K] @ b[N, K]^T).

    b_pretiled: pretile_b(b, glu=act == "swiglu") -- the kernel reads B from it (every DMA one
    contiguous KiB); `b` still gives the shape (kd_gemm_desc.b_pretiled).

    split_k: 0 = library cost model (bounded by the cached GEMM_SPLITK_WS workspace),
    1 = never split, >1 = forced number of K splits (tests).

    `a`/`b` may be K-contiguous tensors or transposed views (x.t() of a contiguous tensor):
    the kernel reads either layout directly (no transpose copies).

    act="swiglu": b = [gate; up] ([2I, K]), out [M, I] = silu(gate) * up, aux (optional)
    the [M, 2I] pre-activation (include/kdstep.h KD_ACT_SWIGLU).

    row_stats: fp32 [M, ceil(N / 256), 8] receives the per-row softmax statistics of the bf16
    output per 256-column tile (kd_gemm_desc.row_stats; the lm_head GEMMs of the KD step).
    """
    if split_k == 0:
        split_k = _SPLIT_DEFAULT[0]
    d, out, M, N, K, la, lb = _gemm_desc(a, b, out, bias, act, residual, aux, alpha, alpha_dev, accumulate,
                                         out_dtype, residual_row_mod, variant, split_k)
    if row_stats is not None:
        _require(row_stats, torch.float32, "row_stats")
        if not row_stats.is_contiguous() or row_stats.numel() != M * ((N + 255) // 256) * 8:
            raise RuntimeError("row_stats: expected a contiguous fp32 [M, ceil(N/256), 8]")
        d.row_stats = row_stats.data_ptr()
        d.row_stats_vs = int(row_stats_vs)
        d.row_stats_inv_t = float(row_stats_inv_t)
        d.row_stats_top2 = 1 if row_stats_top2 else 0
    if b_pretiled is not None:
        _set_pretiled(d, b_pretiled, N, K, act == "swiglu")
    NV.call("kd_gemm", C.byref(d), _stream())
    return out


def _set_pretiled(d, bt, N, K, glu):
    need = NV.lib().kd_gemm_pretile_size(N, K, 1 if glu else 0)
    if not bt.is_contiguous() or bt.numel() * bt.element_size() != need:
        raise RuntimeError(f"b_pretiled: expected a contiguous pretile_b() buffer of {need} bytes")
    d.B = bt.data_ptr()
    d.b_pretiled = 1


def pretile_b(w: torch.Tensor, glu: bool = False) -> torch.Tensor:
    """w [N, K] bf16 (K contiguous) -> the pre-tiled B of kd_gemm_desc.b_pretiled (kd_gemm_pretile):
    each 256-row tile's 32-k stages as the exact LDS images the 256x256 kernel stages; glu: the
    fused SwiGLU GEMM's gate|up row gather (w = [gate; up])."""
    _require(w, torch.bfloat16, "pretile_b.w")
    N, K = w.shape
    if w.stride(1) != 1:
        raise RuntimeError("pretile_b: rows must be K-contiguous")
    n = NV.lib().kd_gemm_pretile_size(N, K, 1 if glu else 0)
    out = torch.empty(n // 2, dtype=torch.bfloat16, device=w.device)
    NV.call("kd_gemm_pretile", w.data_ptr(), w.stride(0), N, K, 1 if glu else 0, out.data_ptr(), _stream())
    return out


# ------------------------------------------------------------------ fp8 path ----
def quant_rows_fp8(x: torch.Tensor, q: torch.Tensor | None = None, scale: torch.Tensor | None = None):
    """bf16 [R, K] -> (e4m3 bytes uint8 [R, K], fp32 scale [R]): per-row amax / 448 scaling
    (kd_quant_rows_fp8; the fp8 teacher's activations and weights)."""
    _require(x, torch.bfloat16, "quant_rows_fp8.x")
    R, K = x.shape
    if x.stride(1) != 1:
        raise RuntimeError("quant_rows_fp8: rows must be contiguous")
    q = q if q is not None else torch.empty((R, K), dtype=torch.uint8, device=x.device)
    scale = scale if scale is not None else torch.empty(R, dtype=torch.float32, device=x.device)
    NV.call("kd_quant_rows_fp8", x.data_ptr(), x.stride(0), R, K, q.data_ptr(), q.stride(0), scale.data_ptr(),
            _stream())
    return q, scale


def gemm_fp8(qa: torch.Tensor, sa: torch.Tensor, qb: torch.Tensor, sb: torch.Tensor, out: torch.Tensor | None = None,
             *, bias=None, act=None, residual=None, aux=None, alpha: float = 1.0) -> torch.Tensor:
    """out[M, N] = epilogue(alpha * sa[m] * sb[n] * qa[M, K] @ qb[N, K]^T), e4m3 operands (uint8
    bytes, K-major), bf16 out (kd_gemm, ab_dtype = KD_DTYPE_FP8_E4M3)."""
    M, K = qa.shape
    N, K2 = qb.shape
    if K != K2 or qa.dtype != torch.uint8 or qb.dtype != torch.uint8:
        raise RuntimeError("gemm_fp8: uint8 (e4m3) operands with equal K")
    if out is None:
        out = torch.empty((M, N // 2 if act == "swiglu" else N), dtype=torch.bfloat16, device=qa.device)
    d = NV.KdGemmDesc()
    d.M, d.N, d.K, d.a_layout, d.b_layout = M, N, K, NV.KD_LAYOUT_K_MAJOR, NV.KD_LAYOUT_K_MAJOR
    d.A, d.lda, d.B, d.ldb = qa.data_ptr(), qa.stride(0), qb.data_ptr(), qb.stride(0)
    d.C, d.ldc, d.c_dtype = out.data_ptr(), out.stride(0), NV.KD_DTYPE_BF16
    d.alpha = float(alpha)
    if bias is not None:
        d.bias, d.bias_dtype = bias.data_ptr(), _DT[bias.dtype]
    d.act = ACTS[act]
    if residual is not None:
        d.residual, d.ldr = residual.data_ptr(), residual.stride(0)
    if aux is not None:
        d.aux, d.ld_aux = aux.data_ptr(), aux.stride(0)
    d.ab_dtype, d.a_scale, d.b_scale = NV.KD_DTYPE_FP8_E4M3, sa.data_ptr(), sb.data_ptr()
    NV.call("kd_gemm", C.byref(d), _stream())
    return out


# ---------------------------------------------------------------- attention ----
def attn_fwd(q, k, v, hd: int, causal: bool, want_lse: bool = True):
    """q [B,H,S,hdp], k/v [B,HKV,S,hdp] bf16 -> (o [B,S,H,hd] bf16, lse [B,H,S] fp32 | None)."""
    B, H, S, hdp = q.shape
    HKV = k.shape[1]
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _require(t, torch.bfloat16, n)
        if not t.is_contiguous():
            raise RuntimeError(f"attn_fwd: {n} must be contiguous")
    o = torch.empty((B, S, H, hd), dtype=torch.bfloat16, device=q.device)
    lse = torch.empty((B, H, S), dtype=torch.float32, device=q.device) if want_lse else None
    d = NV.KdAttnDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), _ptr(lse), B, H, HKV, S, hd, hdp,
                      int(causal))
    NV.call("kd_attn_fwd", C.byref(d), _stream())
    return o, lse


def attn_bwd(q, k, v, o, do, lse, hd: int, causal: bool, dqkv=None, cos=None, sin=None):
    """Returns (dq fp32 [B,H,S,hdp] scaled, dk, dv bf16 [B,HKV,S,hdp]); with `dqkv` (a token-major
    bf16 [B*S, >= (H+2*HKV)*hd] tensor) the three land there directly in qkv_merge's layout (dq and
    dk rotated back with the RoPE tables cos / sin [S, hd/2] when given: GQA, hd == hdp) and that
    tensor is returned instead."""
    B, H, S, hdp = q.shape
    HKV = k.shape[1]
    dev = q.device
    do = do.contiguous()
    delta = _workspace("attn_delta", B * H * S * 4, dev)
    if dqkv is not None:
        _require(dqkv, torch.bfloat16, "attn_bwd.dqkv")
        if dqkv.dim() != 2 or dqkv.stride(1) != 1 or dqkv.shape[0] != B * S or dqkv.shape[1] < (H + 2 * HKV) * hd:
            raise RuntimeError("attn_bwd.dqkv: expected a row-major [B*S, >= (H+2*HKV)*hd] view")
        dq = dk = dv = None
    else:
        dq = torch.empty((B, H, S, hdp), dtype=torch.float32, device=dev)
        dk = torch.empty_like(k)
        dv = torch.empty_like(v)
    d = NV.KdAttnBwdDesc(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                         delta.data_ptr(), _ptr(dq), _ptr(dk), _ptr(dv), B, H, HKV, S, hd, hdp,
                         int(causal), None, 0, _ptr(dqkv), 0 if dqkv is None else dqkv.stride(0), _ptr(cos), _ptr(sin))
    need = NV.lib().kd_attn_bwd_workspace_size(C.byref(d))
    if need:
        ws = _workspace("attn_bwd_partials", need, dev)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
    NV.call("kd_attn_bwd", C.byref(d), _stream())
    return dqkv if dqkv is not None else (dq, dk, dv)


# -------------------------------------------------------------------- norms ----
def norm_fwd(x, weight, bias=None, eps: float = 1e-6, rms: bool = False, out=None, save_stats: bool = True):
    """LayerNorm (rms=False) / RMSNorm (rms=True) over the last dim of a 2-D bf16 or fp32
    (residual stream) tensor; bf16 output."""
    R, D = x.shape
    if x.dtype not in _DT:
        raise RuntimeError("norm_fwd: x must be bf16 or fp32")
    y = out if out is not None else torch.empty((R, D), dtype=torch.bfloat16, device=x.device)
    mean = torch.empty(R, dtype=torch.float32, device=x.device) if (save_stats and not rms) else None
    rstd = torch.empty(R, dtype=torch.float32, device=x.device) if save_stats else None
    NV.call("kd_norm_fwd", int(rms), x.data_ptr(), x.stride(0), weight.data_ptr(), _ptr(bias), y.data_ptr(),
            y.stride(0), _ptr(mean), _ptr(rstd), R, D, float(eps), _DT[x.dtype], _stream())
    return y, mean, rstd


def norm_bwd(x, weight, dy, mean, rstd, dx=None, dx_accum: bool = False, dweight=None, dbias=None,
             accum_w: bool = True, rms: bool = False):
    R, D = x.shape
    if dx is None:
        dx = torch.empty((R, D), dtype=torch.bfloat16, device=x.device)
    nb = NV.lib().kd_norm_bwd_workspace_size(R, D)
    ws = _workspace("norm_bwd", nb, x.device)
    NV.call("kd_norm_bwd", int(rms), x.data_ptr(), x.stride(0), weight.data_ptr(), dy.data_ptr(), dy.stride(0),
            _ptr(mean), rstd.data_ptr(), dx.data_ptr(), dx.stride(0), int(dx_accum), _ptr(dweight), _ptr(dbias),
            int(accum_w), ws.data_ptr(), ws.numel(), R, D, _DT[x.dtype], _stream())
    return dx


# -------------------------------------------------------------- q/k/v, mlp ----
def qkv_split(qkv, B, S, nq, nkv, hd, hdp, cos=None, sin=None):
    dev = qkv.device
    q = torch.empty((B, nq, S, hdp), dtype=torch.bfloat16, device=dev)
    k = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
    v = torch.empty((B, nkv, S, hdp), dtype=torch.bfloat16, device=dev)
    NV.call("kd_qkv_split", qkv.data_ptr(), qkv.stride(0), q.data_ptr(), k.data_ptr(), v.data_ptr(), _ptr(cos),
            _ptr(sin), B, S, nq, nkv, hd, hdp, _stream())
    return q, k, v


def qkv_merge(dq, dk, dv, B, S, nq, nkv, hd, hdp, cos=None, sin=None, out=None):
    if out is None:
        out = torch.empty((B * S, (nq + 2 * nkv) * hd), dtype=torch.bfloat16, device=dq.device)
    NV.call("kd_qkv_merge", dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), out.data_ptr(), out.stride(0), _ptr(cos),
            _ptr(sin), B, S, nq, nkv, hd, hdp, _stream())
    return out


def swiglu_fwd(gu, I: int, out=None):
    M = gu.shape[0]
    h = out if out is not None else torch.empty((M, I), dtype=torch.bfloat16, device=gu.device)
    NV.call("kd_swiglu_fwd", gu.data_ptr(), gu.stride(0), h.data_ptr(), h.stride(0), M, I, _stream())
    return h


def swiglu_bwd(gu, dh, I: int, out=None):
    M = gu.shape[0]
    dgu = out if out is not None else torch.empty((M, 2 * I), dtype=torch.bfloat16, device=gu.device)
    NV.call("kd_swiglu_bwd", gu.data_ptr(), gu.stride(0), dh.data_ptr(), dh.stride(0), dgu.data_ptr(), dgu.stride(0),
            M, I, _stream())
    return dgu


def act_bwd(pre, dy, act: str, out=None):
    dx = out if out is not None else torch.empty_like(dy)
    NV.call("kd_act_bwd", pre.data_ptr(), dy.data_ptr(), dx.data_ptr(), dy.numel(), ACTS[act], _stream())
    return dx


def patchify(pixels, ps: int, kp: int):
    """pixels [NI, 3, img, img] (fp32/bf16) -> [NI*(img/ps)^2, kp] bf16."""
    NI, _, img, _ = pixels.shape
    pixels = pixels.contiguous()
    out = torch.empty((NI * (img // ps) ** 2, kp), dtype=torch.bfloat16, device=pixels.device)
    NV.call("kd_patchify", pixels.data_ptr(), _DT[pixels.dtype], out.data_ptr(), NI, img, ps, kp, _stream())
    return out


def embed_assemble(ids, src, table, feats, newline, err):
    M = ids.numel()
    H = table.shape[1]
    out = torch.empty((M, H), dtype=torch.bfloat16, device=ids.device)
    NV.call("kd_embed_assemble", ids.data_ptr(), src.data_ptr(), table.data_ptr(), _ptr(feats), _ptr(newline),
            out.data_ptr(), M, H, table.shape[0], err.data_ptr(), _stream())
    return out


def embed_bwd(ids, src, dout, dtable=None, dfeats=None, dnewline=None):
    M, H = dout.shape
    NV.call("kd_embed_bwd", ids.data_ptr(), src.data_ptr(), dout.data_ptr(), _ptr(dtable), _ptr(dfeats),
            _ptr(dnewline), M, H, _stream())


def colsum(dy, out, accumulate: bool = True):
    M, Nn = dy.shape
    NV.call("kd_colsum", dy.data_ptr(), dy.stride(0), M, Nn, out.data_ptr(), int(accumulate), _stream())
    return out


def row_group_mean(x, G: int, P: int):
    D = x.shape[1]
    out = torch.empty((G, D), dtype=torch.float32, device=x.device)
    NV.call("kd_row_group_mean", x.data_ptr(), x.stride(0), G, P, D, out.data_ptr(), _stream())
    return out


def row_group_mean_bwd(dpool, P: int, out=None, scale_dev=None):
    G, D = dpool.shape
    if out is None:
        out = torch.empty((G * P, D), dtype=torch.bfloat16, device=dpool.device)
    NV.call("kd_row_group_mean_bwd", dpool.data_ptr(), G, P, D, out.data_ptr(), out.stride(0), _ptr(scale_dev),
            _stream())
    return out


def ntxent(fs, ft, tau: float = 0.07, weight: float = 1.0, want_grad: bool = True, grad_scale: float = 1.0,
           loss_out=None, dfs_out=None):
    """fs/ft: pooled features [n, D] fp32.  Returns (loss2 [weighted, raw], dfs | None)."""
    n, D = fs.shape
    loss = loss_out if loss_out is not None else torch.empty(2, dtype=torch.float32, device=fs.device)
    dfs = (dfs_out if dfs_out is not None else torch.empty_like(fs)) if want_grad else None
    NV.call("kd_ntxent", fs.contiguous().data_ptr(), ft.contiguous().data_ptr(), n, D, float(tau), float(weight),
            loss.data_ptr(), _ptr(dfs), float(grad_scale), _stream())
    return loss, dfs


def adamw(p, pb, g, m, v, lr, b1, b2, eps, wd, step, gscale=None, skip_words=None):
    """skip_words: optional int32 device tensor; any nonzero word makes the step a no-op."""
    ns = 0 if skip_words is None else skip_words.numel()
    NV.call("kd_adamw", p.data_ptr(), pb.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), float(lr),
            float(b1), float(b2), float(eps), float(wd), int(step), _ptr(gscale), _ptr(skip_words), ns, _stream())


def zero_(x: torch.Tensor) -> torch.Tensor:
    """x[...] = 0 on the current stream through the library (kd_zero; x contiguous)."""
    if not x.is_contiguous():
        raise RuntimeError("zero_: needs a contiguous tensor")
    NV.call("kd_zero", x.data_ptr(), x.numel() * x.element_size(), _stream())
    return x


def sumsq(x, out):
    NV.call("kd_sumsq", x.data_ptr(), x.numel(), out.data_ptr(), _stream())
    return out


def scale_f32(x, s_dev=None, out=None):
    """out = x * s_dev (a device fp32 scalar; None: a copy), fp32 (kd_scale_f32)."""
    _require(x, torch.float32, "scale_f32.x")
    if out is None:
        out = torch.empty_like(x)
    NV.call("kd_scale_f32", x.data_ptr(), _ptr(s_dev), out.data_ptr(), x.numel(), _stream())
    return out


def scalar_mul(a, b, out=None):
    """out = a * b elementwise on device fp32 scalars (kd_scalar_mul)."""
    _require(a, torch.float32, "a")
    _require(b, torch.float32, "b")
    if a.numel() != b.numel():
        raise RuntimeError("scalar_mul: size mismatch")
    out = out if out is not None else torch.empty_like(a)
    NV.call("kd_scalar_mul", a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), _stream())
    return out


def cast_f32_bf16(x, y):
    NV.call("kd_cast_f32_bf16", x.data_ptr(), y.data_ptr(), x.numel(), _stream())
    return y


def cast_bf16_f32(x, y):
    NV.call("kd_cast_bf16_f32", x.data_ptr(), y.data_ptr(), x.numel(), _stream())
    return y


def image_src_map(ids, image_token: int, maps, map_len, err):
    """ids [B, L] int64 -> src int32 [B*L] (see include/kdstep.h kd_image_src_map)."""
    B, L = ids.shape
    src = torch.empty(B * L, dtype=torch.int32, device=ids.device)
    NV.call("kd_image_src_map", ids.contiguous().data_ptr(), B, L, int(image_token), maps.data_ptr(), maps.shape[1],
            map_len.data_ptr(), src.data_ptr(), err.data_ptr(), _stream())
    return src


_DEPTH_DTYPES = {torch.uint16: 0, torch.int32: 1, torch.float32: 2}


def depth_to_3ch(depth: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """depth [B, H, W] or [H, W] (uint16 / int32 / float32, device) -> uint8 [..., H, W, 3]
    (kd_depth_to_3ch: normalised depth, Prewitt magnitude, Prewitt angle; each image
    normalised by its own range)."""
    if not depth.is_cuda:
        raise RuntimeError("depth_to_3ch: expected a device tensor (no CPU path)")
    if depth.dtype not in _DEPTH_DTYPES:
        raise RuntimeError(f"depth_to_3ch: dtype {depth.dtype} not in uint16/int32/float32")
    if depth.dim() not in (2, 3):
        raise RuntimeError(f"depth_to_3ch: expected [H, W] or [B, H, W], got {tuple(depth.shape)}")
    d = depth.contiguous()
    B, H, W = (1, *d.shape) if d.dim() == 2 else d.shape
    if out is None:
        out = torch.empty((*d.shape, 3), dtype=torch.uint8, device=d.device)
    elif out.shape != (*d.shape, 3) or out.dtype != torch.uint8 or not out.is_contiguous():
        raise RuntimeError("depth_to_3ch: out must be a contiguous uint8 [..., H, W, 3] tensor")
    nbytes = NV.lib().kd_depth_to_3ch_workspace_size(B, H, W)
    ws = _workspace(("depth3", _stream()), nbytes, d.device)
    NV.call("kd_depth_to_3ch", d.data_ptr(), _DEPTH_DTYPES[d.dtype], B, H, W, out.data_ptr(), ws.data_ptr(),
            ws.numel(), _stream())
    return out


def image_resize_u8(img: torch.Tensor, out_h: int, out_w: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """[H, W, 3] uint8 (device) -> [out_h, out_w, 3] uint8: PIL Image.resize(BICUBIC), bit-exact
    (kd_image_resize_u8)."""
    _require(img, torch.uint8, "image_resize_u8")
    if img.dim() != 3 or img.shape[2] != 3:
        raise RuntimeError(f"image_resize_u8: expected [H, W, 3], got {tuple(img.shape)}")
    x = img.contiguous()
    H, W = int(x.shape[0]), int(x.shape[1])
    if out is None:
        out = torch.empty((out_h, out_w, 3), dtype=torch.uint8, device=x.device)
    nbytes = NV.lib().kd_image_resize_workspace_size(H, W, out_h, out_w)
    ws = _workspace(("image_resize", _stream()), nbytes, x.device)
    NV.call("kd_image_resize_u8", x.data_ptr(), H, W, out.data_ptr(), int(out_h), int(out_w), ws.data_ptr(),
            ws.numel(), _stream())
    return out


def anyres_tiles(base: torch.Tensor, resized: torch.Tensor, best_hw, n_out: int, mean, std,
                 dtype=torch.float32, patch: int = 384, out: torch.Tensor | None = None) -> torch.Tensor:
    """pixel_values [n_out, 3, patch, patch] of one image from its base resize and its
    aspect-preserving resize (kd_anyres_tiles)."""
    _require(base, torch.uint8, "anyres_tiles")
    _require(resized, torch.uint8, "anyres_tiles")
    if dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError(f"anyres_tiles: dtype {dtype} not float32/bfloat16")
    if tuple(base.shape) != (patch, patch, 3):
        raise RuntimeError(f"anyres_tiles: base must be [{patch}, {patch}, 3], got {tuple(base.shape)}")
    bh, bw = int(best_hw[0]), int(best_hw[1])
    nh, nw = int(resized.shape[0]), int(resized.shape[1])
    if out is None:
        out = torch.empty((n_out, 3, patch, patch), dtype=dtype, device=base.device)
    ms = (C.c_float * 6)(*[float(v) for v in mean], *[float(v) for v in std])
    NV.call("kd_anyres_tiles", base.contiguous().data_ptr(), resized.contiguous().data_ptr(), nh, nw, bh, bw, patch,
            int(n_out), C.cast(ms, C.c_void_p), out.data_ptr(), 0 if dtype == torch.float32 else 1, _stream())
    return out


def attn_decode(q: torch.Tensor, k_new: torch.Tensor, v_new: torch.Tensor, k_cache: torch.Tensor,
                v_cache: torch.Tensor, n: int, hd: int, cur: torch.Tensor | None = None,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """One token's attention against cache positions [0, n) (kd_attn_decode); the token's own
    k_new/v_new [HKV, hdp] are stored at position n - 1.  n = cur[0] (device int32) when given.
    q [H, hdp], caches [HKV, smax, hdp] bf16 -> o [1, H*hd] bf16 (token-major, what o_proj reads)."""
    H, hdp = q.shape
    HKV, smax, _ = k_cache.shape
    if out is None:
        out = torch.empty((1, H * hd), dtype=torch.bfloat16, device=q.device)
    nbytes = NV.lib().kd_attn_decode_workspace_size(H, hd, smax)
    ws = _workspace(("attn_decode", _stream()), nbytes, q.device)
    NV.call("kd_attn_decode", q.data_ptr(), k_new.data_ptr(), v_new.data_ptr(), k_cache.data_ptr(),
            v_cache.data_ptr(), out.data_ptr(), H, HKV, hd, hdp, smax, int(n), _ptr(cur), ws.data_ptr(), ws.numel(),
            _stream())
    return out


def gemv(x: torch.Tensor, w: torch.Tensor, *, bias=None, residual=None, swiglu_inter: int = 0, norm_w=None,
         eps: float = 1e-6) -> torch.Tensor:
    """One token row through a linear layer (kd_gemv): x [1, K] bf16, w [N, K] (row stride may
    exceed K) -> [1, N] bf16 with an optional bias / residual / SwiGLU (w = gate|up, N = 2*inter),
    and with norm_w the RMSNorm of x fused in front."""
    K = x.shape[-1]
    epi, extra = 0, None
    if swiglu_inter:
        epi, N = 3, int(swiglu_inter)
    else:
        N = w.shape[0]
        if bias is not None:
            epi, extra = 1, bias
        elif residual is not None:
            epi, extra = 2, residual
    y = torch.empty((1, N), dtype=torch.bfloat16, device=x.device)
    NV.call("kd_gemv", x.data_ptr(), w.data_ptr(), w.stride(0), _ptr(extra), y.data_ptr(), N, K, epi,
            int(swiglu_inter), _ptr(norm_w), float(eps), _stream())
    return y


def gen_select(logits: torch.Tensor, seq: torch.Tensor, length: int, repetition_penalty: float = 1.0,
               no_repeat_ngram_size: int = 0, out: torch.Tensor | None = None, cur: torch.Tensor | None = None) -> None:
    """Greedy next token of one bf16 logits row with the repetition-penalty / no-repeat-n-gram
    processors; written to seq[length] (length = cur[0], then incremented, when cur is given)
    (kd_gen_select)."""
    V = logits.shape[-1]
    ws = _workspace(("gen_select", _stream()), V, logits.device)
    NV.call("kd_gen_select", logits.data_ptr(), V, seq.data_ptr(), int(length), _ptr(cur), float(repetition_penalty),
            int(no_repeat_ngram_size), ws.data_ptr(), ws.numel(), _ptr(out), _stream())


def rope_row(cos: torch.Tensor, sin: torch.Tensor, cur: torch.Tensor, cos_row: torch.Tensor, sin_row: torch.Tensor):
    """cos/sin row of position cur[0] - 1 into the one-row buffers (kd_rope_row)."""
    NV.call("kd_rope_row", cos.data_ptr(), sin.data_ptr(), cos.shape[1], cur.data_ptr(), cos_row.data_ptr(),
            sin_row.data_ptr(), _stream())
