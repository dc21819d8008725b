"""ctypes binding of the C-ABI library libkdstep.so (include/kdstep.h).

This is the exact binding a maintainer of the reference would add: plain pointers,
sizes and an int status per call.  A non-zero status raises RuntimeError with the
library's thread-local message (mirroring the reference's RuntimeError behaviour).

There is NO fallback: if the library is missing the import of any op fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("KDSTEP_LIB", _PKG / "libkdstep.so"))
HEADER = _PKG.parent / "include" / "kdstep.h"

KD_OK = 0
ABI_VERSION = 9
STATUS_NAMES = {
    0: "KD_OK", 1: "KD_ERR_SHAPE", 2: "KD_ERR_DTYPE", 3: "KD_ERR_ALIGN", 4: "KD_ERR_ARCH",
    5: "KD_ERR_LABEL_RANGE", 6: "KD_ERR_LAUNCH", 7: "KD_ERR_ARG", 8: "KD_ERR_WORKSPACE",
}

# kd_loss_variant
KD_LOSS_NONE, KD_LOSS_LOCA, KD_LOSS_KL, KD_LOSS_KL_LOGTARGET = 0, 1, 2, 3


class KdLossParams(C.Structure):
    _fields_ = [
        ("variant", C.c_int32),
        ("temperature", C.c_float),
        ("alpha", C.c_float),
        ("kd_weight", C.c_float),
        ("ce_weight", C.c_float),
        ("grad_scale", C.c_float),
        ("clamp_min", C.c_float),
        ("teacher_ce", C.c_int32),
        ("out_scale", C.c_float),
        ("out_accumulate", C.c_int32),
        ("err_out", C.c_void_p),
        ("row_base", C.c_int32),
        ("dscale", C.c_void_p),
        ("dscale_given", C.c_int32),
        ("s_row_stats", C.c_void_p),
        ("t_row_stats", C.c_void_p),
        ("s_stats", C.c_void_p),
        ("loca_path", C.c_int32),
        ("rr_poll_us_p1", C.c_int32),
        ("standin_count", C.c_void_p),
    ]


# kd_fp8_family
KD_FP8_VISION, KD_FP8_PROJECTOR, KD_FP8_LM_ATTN, KD_FP8_LM_MLP, KD_FP8_LM_HEAD, KD_FP8_ALL = 1, 2, 4, 8, 16, 31

# kd_layout / kd_dtype / kd_act
KD_LAYOUT_K_MAJOR, KD_LAYOUT_MN_MAJOR = 0, 1
KD_DTYPE_BF16, KD_DTYPE_F32, KD_DTYPE_FP8_E4M3 = 0, 1, 2
KD_ACT_NONE, KD_ACT_GELU_TANH, KD_ACT_GELU_ERF, KD_ACT_SILU, KD_ACT_SWIGLU = 0, 1, 2, 3, 4
KD_ACT_DGELU_TANH, KD_ACT_DSWIGLU = 5, 6


class KdGemmDesc(C.Structure):
    _fields_ = [
        ("M", C.c_int32), ("N", C.c_int32), ("K", C.c_int32),
        ("a_layout", C.c_int32), ("b_layout", C.c_int32),
        ("A", C.c_void_p), ("lda", C.c_int64),
        ("B", C.c_void_p), ("ldb", C.c_int64),
        ("C", C.c_void_p), ("ldc", C.c_int64),
        ("c_dtype", C.c_int32), ("accumulate", C.c_int32),
        ("alpha", C.c_float), ("alpha_dev", C.c_void_p),
        ("bias", C.c_void_p), ("bias_dtype", C.c_int32), ("act", C.c_int32),
        ("residual", C.c_void_p), ("ldr", C.c_int64),
        ("aux", C.c_void_p), ("ld_aux", C.c_int64),
        ("residual_row_mod", C.c_int32),
        ("variant", C.c_int32),
        ("split_k", C.c_int32), ("workspace", C.c_void_p), ("workspace_bytes", C.c_uint64),
        ("ab_dtype", C.c_int32), ("a_scale", C.c_void_p), ("b_scale", C.c_void_p),
        ("residual_dtype", C.c_int32),
        ("qkv", C.c_void_p),
        ("row_stats", C.c_void_p), ("row_stats_vs", C.c_int32), ("row_stats_inv_t", C.c_float),
        ("row_stats_top2", C.c_int32),
        ("b_pretiled", C.c_int32),
    ]


class KdQkvScatter(C.Structure):
    _fields_ = [("q", C.c_void_p), ("k", C.c_void_p), ("v", C.c_void_p), ("cos_t", C.c_void_p), ("sin_t", C.c_void_p),
                ("S", C.c_int32), ("nq", C.c_int32), ("nkv", C.c_int32), ("hd", C.c_int32), ("hdp", C.c_int32)]


class KdAttnDesc(C.Structure):
    _fields_ = [("q", C.c_void_p), ("k", C.c_void_p), ("v", C.c_void_p), ("o", C.c_void_p), ("lse", C.c_void_p),
                ("B", C.c_int32), ("H", C.c_int32), ("HKV", C.c_int32), ("S", C.c_int32), ("hd", C.c_int32),
                ("hdp", C.c_int32), ("causal", C.c_int32)]


class KdAttnBwdDesc(C.Structure):
    _fields_ = [("q", C.c_void_p), ("k", C.c_void_p), ("v", C.c_void_p), ("o", C.c_void_p), ("dO", C.c_void_p),
                ("lse", C.c_void_p), ("delta", C.c_void_p), ("dq", C.c_void_p), ("dk", C.c_void_p),
                ("dv", C.c_void_p),
                ("B", C.c_int32), ("H", C.c_int32), ("HKV", C.c_int32), ("S", C.c_int32), ("hd", C.c_int32),
                ("hdp", C.c_int32), ("causal", C.c_int32), ("workspace", C.c_void_p), ("workspace_bytes", C.c_uint64),
                ("dqkv", C.c_void_p), ("ld_qkv", C.c_int64), ("cos_t", C.c_void_p), ("sin_t", C.c_void_p)]


class KdModelConfig(C.Structure):
    _fields_ = [("v_hidden", C.c_int32), ("v_inter", C.c_int32), ("v_layers", C.c_int32), ("v_heads", C.c_int32),
                ("v_patch", C.c_int32), ("v_image", C.c_int32), ("v_eps", C.c_float),
                ("t_hidden", C.c_int32), ("t_inter", C.c_int32), ("t_layers", C.c_int32), ("t_heads", C.c_int32),
                ("t_kv_heads", C.c_int32), ("t_head_dim", C.c_int32), ("t_vocab", C.c_int32), ("t_tie", C.c_int32),
                ("t_rope_theta", C.c_float), ("t_eps", C.c_float),
                ("image_token_id", C.c_int64), ("projector_act", C.c_int32)]


# void (*kd_layer_cb)(void* user, int layer)
LAYER_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int)


class KdError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn}: {STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


_vp, _i32, _i64, _sz, _f32 = C.c_void_p, C.c_int, C.c_int64, C.c_size_t, C.c_float

# name -> (restype, argtypes).  Kept in the same order as include/kdstep.h.
SIGNATURES = {
    "kd_abi_version": (_i32, []),
    "kd_last_error": (C.c_char_p, []),
    "kd_device_is_gfx950": (_i32, [_i32]),
    "kd_loss_workspace_size": (_sz, [_i32, _i32, _i32]),
    "kd_loss_fwd_bwd": (_i32, [_vp, _i64, _i32, _vp, _i64, _i32, _vp, _i32, _i32, KdLossParams,
                               _vp, _vp, _i64, _vp, _sz, _vp]),
    "kd_loss_check": (_i32, [_vp, _vp]),
    "kd_loss_student_stats": (_i32, [_vp, _i64, _i32, _i32, _f32, _vp, _vp]),
    "kd_gemm": (_i32, [C.POINTER(KdGemmDesc), _vp]),
    "kd_gemm_pretile_size": (_sz, [_i32, _i32, _i32]),
    "kd_gemm_pretile": (_i32, [_vp, _i64, _i32, _i32, _i32, _vp, _vp]),
    "kd_attn_fwd": (_i32, [C.POINTER(KdAttnDesc), _vp]),
    "kd_attn_bwd": (_i32, [C.POINTER(KdAttnBwdDesc), _vp]),
    "kd_attn_bwd_workspace_size": (C.c_size_t, [C.POINTER(KdAttnBwdDesc)]),
    "kd_gemm_workspace_size": (C.c_size_t, [C.POINTER(KdGemmDesc)]),
    "kd_gemm_plan": (_i32, [C.POINTER(KdGemmDesc), C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32)]),
    "kd_norm_fwd": (_i32, [_i32, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _vp, _i32, _i32, _f32, _i32, _vp]),
    "kd_norm_bwd_workspace_size": (_sz, [_i32, _i32]),
    "kd_norm_bwd": (_i32, [_i32, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _sz,
                           _i32, _i32, _i32, _vp]),
    "kd_qkv_split": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
    "kd_qkv_merge": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
    "kd_swiglu_fwd": (_i32, [_vp, _i64, _vp, _i64, _i32, _i32, _vp]),
    "kd_swiglu_bwd": (_i32, [_vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _vp]),
    "kd_act_bwd": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp]),
    "kd_patchify": (_i32, [_vp, _i32, _vp, _i32, _i32, _i32, _i32, _vp]),
    "kd_embed_assemble": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    "kd_image_src_map": (_i32, [_vp, _i32, _i32, _i64, _vp, _i32, _vp, _vp, _vp, _vp]),
    "kd_embed_bwd": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp]),
    "kd_colsum": (_i32, [_vp, _i64, _i32, _i32, _vp, _i32, _vp]),
    "kd_row_group_mean": (_i32, [_vp, _i64, _i32, _i32, _i32, _vp, _vp]),
    "kd_row_group_mean_bwd": (_i32, [_vp, _i32, _i32, _i32, _vp, _i64, _vp, _vp]),
    "kd_ntxent": (_i32, [_vp, _vp, _i32, _i32, _f32, _f32, _vp, _vp, _f32, _vp]),
    "kd_adamw": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _f32, _f32, _f32, _f32, _f32, _i32, _vp, _vp, _i32, _vp]),
    "kd_scalar_mul": (_i32, [_vp, _vp, _vp, _i32, _vp]),
    "kd_scale_f32": (_i32, [_vp, _vp, _vp, C.c_int64, _vp]),
    "kd_sumsq": (_i32, [_vp, _i64, _vp, _vp]),
    "kd_zero": (_i32, [_vp, C.c_uint64, _vp]),
    "kd_cast_f32_bf16": (_i32, [_vp, _vp, _i64, _vp]),
    "kd_prefetch": (_i32, [_vp, C.c_uint64, _i32, _vp]),
    "kd_cast_bf16_f32": (_i32, [_vp, _vp, _i64, _vp]),
    "kd_quant_rows_fp8": (_i32, [_vp, _i64, _i32, _i32, _vp, _i64, _vp, _vp]),
    "kd_depth_to_3ch_workspace_size": (_sz, [_i32, _i32, _i32]),
    "kd_depth_to_3ch": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _vp, _sz, _vp]),
    "kd_image_resize_workspace_size": (_sz, [_i32, _i32, _i32, _i32]),
    "kd_attn_decode_workspace_size": (_sz, [_i32, _i32, _i32]),
    "kd_attn_decode": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _sz, _vp]),
    "kd_gemv": (_i32, [_vp, _vp, _i64, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _f32, _vp]),
    "kd_gen_select": (_i32, [_vp, _i32, _vp, _i32, _vp, _f32, _i32, _vp, _sz, _vp, _vp]),
    "kd_rope_row": (_i32, [_vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "kd_image_resize_u8": (_i32, [_vp, _i32, _i32, _vp, _i32, _i32, _vp, _sz, _vp]),
    "kd_anyres_tiles": (_i32, [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _vp]),
    "kd_anyres_batch_map": (_i32, [_vp, _i32, _i32, _vp, _i32, _vp]),
    "kd_model_param_count": (_i32, [C.POINTER(KdModelConfig)]),
    "kd_model_param_numel": (_i64, [C.POINTER(KdModelConfig)]),
    "kd_model_param_info": (_i32, [C.POINTER(KdModelConfig), _i32, C.c_char_p, _i32, C.POINTER(_i64),
                                   C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64)]),
    "kd_model_create": (_i32, [C.POINTER(KdModelConfig), _vp, _vp, C.POINTER(_vp)]),
    "kd_model_destroy": (None, [_vp]),
    "kd_model_set_trainable": (_i32, [_vp, _i32, _i32, _i32]),
    "kd_model_set_residual_f32": (_i32, [_vp, _i32, _i32]),
    "kd_model_fp8_scale_count": (_i64, [_vp]),
    "kd_model_quantize_fp8": (_i32, [_vp, _vp, _vp, _vp]),
    "kd_model_set_fp8": (_i32, [_vp, _vp, _vp]),
    "kd_model_set_fp8_families": (_i32, [_vp, _i32]),
    "kd_model_set_row_stats": (_i32, [_vp, _vp, _i32, _f32, _i32]),
    "kd_model_forward_workspace_size": (_sz, [_vp, _i32, _i32, _i32, _i32]),
    "kd_model_forward": (_i32, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _sz, _vp, _vp, _vp,
                                _vp, _vp, _vp, _vp]),
    "kd_model_backward_workspace_size": (_sz, [_vp, _i32, _i32, _i32]),
    "kd_model_backward": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _sz, _vp, _vp,
                                 LAYER_CB, _vp]),
    "kd_timer_enable": (None, [_i32]),
    "kd_timer_count": (_i32, []),
    "kd_timer_read": (_i32, [_i32, C.c_char_p, _i32, C.POINTER(C.c_double), C.POINTER(_f32)]),
    "kd_timer_reset": (None, []),
}

_lib = None


def lib() -> C.CDLL:
    """Load libkdstep.so once.  Raises if it is missing (no silent fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(
                f"libkdstep.so not found at {LIB_PATH}; run `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (hipcc --offload-arch=gfx950)")
        l = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        if l.kd_abi_version() != ABI_VERSION:
            raise ImportError("libkdstep.so ABI version mismatch")
        _lib = l
    return _lib


def check(fn: str, status: int) -> None:
    if status != KD_OK:
        msg = lib().kd_last_error().decode(errors="replace")
        raise KdError(fn, status, msg)


def call(fn: str, *args) -> None:
    check(fn, getattr(lib(), fn)(*args))


def header_symbols() -> list[str]:
    """Function names declared in include/kdstep.h (for the export test)."""
    import re
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(kd_[a-z0-9_]+)\s*\(", txt, flags=re.M)
    return sorted(set(names))
