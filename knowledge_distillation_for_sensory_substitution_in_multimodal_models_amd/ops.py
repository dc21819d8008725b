"""Python-side launchers of the C-ABI kernels (device tensors in, device tensors out).

PyTorch is plumbing here: it allocates device memory and provides the stream; every
FLOP runs in libkdstep.so.  There is no CPU or torch fallback for any op.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _native as N

_WS: dict = {}


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
VARIANTS = {"none": N.KD_LOSS_NONE, "loca": N.KD_LOSS_LOCA, "kl": N.KD_LOSS_KL,
            "kl_logtarget": N.KD_LOSS_KL_LOGTARGET}


def kd_loss_fwd_bwd(student_logits: torch.Tensor, teacher_logits: torch.Tensor | None,
                    labels: torch.Tensor, variant: str, temperature: float = 1.0, alpha: float = 0.8,
                    kd_weight: float = 1.0, ce_weight: float = 1.0, grad_scale: float = 1.0,
                    clamp_min: float = 1e-8, teacher_ce: bool = True, want_grad: bool = True,
                    check: bool = False):
    """Fused KD-loss forward + backward (include/kdstep.h kd_loss_fwd_bwd).

    student_logits [B, L, V_s] bf16 (last dim contiguous), teacher_logits [B, L, V_t] bf16,
    labels [B, L] int64.  Returns (loss4, dlogits): loss4 = fp32 [4] =
    (kd_term, student_ce, teacher_ce, total); dlogits bf16 [B, L, V_s] or None.
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
        if v != N.KD_LOSS_NONE:
            raise RuntimeError(f"kd_loss variant {variant} needs teacher logits")
        V_t, ld_t = 0, 0
    dev = student_logits.device
    loss = torch.empty(4, dtype=torch.float32, device=dev)
    dl = torch.empty((B, L, V_s), dtype=torch.bfloat16, device=dev) if want_grad else None
    nbytes = N.lib().kd_loss_workspace_size(B, L, V_s)
    ws = _workspace("kd_loss", nbytes, dev)
    prm = N.KdLossParams(v, float(temperature), float(alpha), float(kd_weight), float(ce_weight),
                         float(grad_scale), float(clamp_min), 1 if teacher_ce else 0)
    N.call("kd_loss_fwd_bwd", _ptr(teacher_logits), ld_t, V_t, _ptr(student_logits),
           student_logits.stride(1), V_s, _ptr(labels), B, L, prm, _ptr(loss), _ptr(dl),
           V_s, _ptr(ws), ws.numel(), _stream())
    if check:
        N.call("kd_loss_check", _ptr(ws), _stream())
    return loss, dl


# --------------------------------------------------------------------- GEMM ----
ACTS = {None: N.KD_ACT_NONE, "none": N.KD_ACT_NONE, "gelu_tanh": N.KD_ACT_GELU_TANH,
        "gelu_erf": N.KD_ACT_GELU_ERF, "silu": N.KD_ACT_SILU}
_DT = {torch.bfloat16: N.KD_DTYPE_BF16, torch.float32: N.KD_DTYPE_F32}


def _operand(x: torch.Tensor, name: str):
    """(ptr, ld, layout, rows, k) of a 2-D bf16 operand; MN-major if it is a transposed view."""
    _require(x, torch.bfloat16, name)
    if x.dim() != 2:
        raise RuntimeError(f"{name}: expected 2-D")
    r, k = x.shape
    if x.stride(1) == 1 and (x.stride(0) >= k or r == 1):
        return x.data_ptr(), max(x.stride(0), k), N.KD_LAYOUT_K_MAJOR
    if x.stride(0) == 1 and (x.stride(1) >= r or k == 1):
        return x.data_ptr(), max(x.stride(1), r), N.KD_LAYOUT_MN_MAJOR
    raise RuntimeError(f"{name}: needs a unit stride in one dimension")


def gemm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, *, bias=None, act=None,
         residual=None, aux=None, alpha: float = 1.0, alpha_dev=None, accumulate: bool = False,
         out_dtype=torch.bfloat16) -> torch.Tensor:
    """out[M, N] = epilogue(alpha * a[M, K] @ b[N, K]^T).

    `a`/`b` may be K-contiguous tensors or transposed views (x.t() of a contiguous tensor):
    the kernel reads either layout directly (no transpose copies).
    """
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise RuntimeError(f"gemm: K mismatch {K} vs {K2}")
    pa, lda, la = _operand(a, "gemm.a")
    pb, ldb, lb = _operand(b, "gemm.b")
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=a.device)
    if out.stride(1) != 1:
        raise RuntimeError("gemm: out must have a contiguous last dim")
    d = N.KdGemmDesc()
    d.M, d.N, d.K, d.a_layout, d.b_layout = M, N, K, la, lb
    d.A, d.lda, d.B, d.ldb = pa, lda, pb, ldb
    d.C, d.ldc, d.c_dtype, d.accumulate = out.data_ptr(), out.stride(0), _DT[out.dtype], int(accumulate)
    d.alpha, d.alpha_dev = float(alpha), _ptr(alpha_dev)
    if bias is not None:
        d.bias, d.bias_dtype = bias.data_ptr(), _DT[bias.dtype]
    d.act = ACTS[act]
    if residual is not None:
        _require(residual, torch.bfloat16, "gemm.residual")
        d.residual, d.ldr = residual.data_ptr(), residual.stride(0)
    if aux is not None:
        _require(aux, torch.bfloat16, "gemm.aux")
        d.aux, d.ld_aux = aux.data_ptr(), aux.stride(0)
    N.call("kd_gemm", C.byref(d), _stream())
    return out
