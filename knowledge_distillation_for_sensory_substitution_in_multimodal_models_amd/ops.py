"""Python-side launchers of the C-ABI kernels (device tensors in, device tensors out).

PyTorch is plumbing here: it allocates device memory and provides the stream; every
FLOP runs in libkdstep.so.  There is no CPU or torch fallback for any op.
"""
from __future__ import annotations

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
