"""ctypes binding of libstcgan_hip.so (C-ABI: include/stcgan_hip.h).

The library is built in-tree (``shadow-removal-istd_amd/csrc/Makefile``) and
loaded from this directory.  There is no fallback: if the library is missing
or a call fails, a RuntimeError is raised.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STC_LIB_PATH") or os.path.join(_HERE, "libstcgan_hip.so")  # override: A/B timing

F32, BF16 = 0, 1
CONV_S2, CONV_S1, CONVT_S2, CONV_S1_DGRAD = 0, 1, 2, 3
PACK_CONV_FWD, PACK_CONV_DGRAD, PACK_CONV_S1_DGRAD, PACK_CONVT_FWD, PACK_CONVT_DGRAD = 0, 1, 2, 3, 4
LOSS_L1, LOSS_MSE_CONST, LOSS_BCE_CONST = 0, 1, 2
LOSS_COMBINE_D, LOSS_COMBINE_G = 0, 1


class View(ctypes.Structure):
    """stc_view: element (b, y, x, c) at p + b*bs + y*rs + x*ps + (co + c)*cs."""
    _fields_ = [("p", ctypes.c_void_p), ("H", ctypes.c_int32), ("W", ctypes.c_int32),
                ("bs", ctypes.c_int64), ("rs", ctypes.c_int64), ("ps", ctypes.c_int32),
                ("co", ctypes.c_int32), ("cs", ctypes.c_int32), ("pad_", ctypes.c_int32)]


NULL_VIEW = View(None, 0, 0, 0, 0, 0, 0, 1, 0)

PACK_MAX = 40


class BnbFuse(ctypes.Structure):
    """stc_bnb_fuse: the BatchNorm-backward reduction fused into an input-gradient conv."""
    _fields_ = [("x", View), ("g_other", View), ("scale", ctypes.c_void_p), ("shift", ctypes.c_void_p),
                ("mean", ctypes.c_void_p), ("rstd", ctypes.c_void_p), ("slope_self", ctypes.c_float),
                ("slope_other", ctypes.c_float), ("C", ctypes.c_int32), ("ch_off", ctypes.c_int32)]


class PackDesc(ctypes.Structure):
    """stc_pack_desc: one stc_pack_weight job of a multi-tensor stc_pack_weights launch."""
    _fields_ = [("mode", ctypes.c_int32), ("P", ctypes.c_int32), ("Q", ctypes.c_int32), ("N_pad", ctypes.c_int32),
                ("C_pad", ctypes.c_int32), ("pad_", ctypes.c_int32), ("W", ctypes.c_void_p), ("out", ctypes.c_void_p)]

_vp, _i32, _i64, _f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float

# name: (restype, argtypes)
_SIGS = {
    "stc_conv_fwd": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _vp, _i32, _f32, _vp, _i32, View, _vp, _i32, _i32,
                            _vp, _i64, _vp]),
    "stc_conv_fwd_workspace": (_i64, [_i32, _i32, _i32, _i32, _i32, _i32, _i32]),
    "stc_conv_fwd_plan": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp]),
    "stc_conv_fwd_query": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "stc_conv_bwd_bn_chunks": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32]),
    "stc_conv_bwd_bn_chunks_ex": (_i32, [_i32, _i32, _i32, View, _i32, _i32, View, _vp]),
    "stc_conv_bwd_bn": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _i32, View, _vp, _vp, _i32, _vp, _i64, _vp]),
    "stc_conv_fwd_ex": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _i32, View, _vp, _i32, _i32, _vp, _i32, _vp, _vp,
                               _i64, _vp]),
    "stc_conv_fwd_act_ok": (_i32, [_i32, _i32, _i32, View, _i32, _i32, View, View]),
    "stc_conv_fwd_act": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _i32, View, _f32, View, _f32, _vp, _vp, _i64, _vp]),
    "stc_conv_bwd_bn_apply": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _i32, View, _vp, _vp, _i32, _vp, View, _vp,
                                     _vp, _vp, _i64, _vp]),
    "stc_conv_bn_fwd": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _i32, View, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _f32,
                               _f32, View, View, _f32, View, _f32, _vp, _i64, _vp]),
    "stc_conv_bwd_act_ok": (_i32, [_i32, _i32, _i32, View, _i32, _i32, View, View, View]),
    "stc_conv_bwd_act": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _i32, View, View, _f32, View, _f32, _vp]),
    "stc_set_splitk_inlaunch": (_i32, [_i32]),
    "stc_conv_wgrad": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _vp, _i32, _f32, View, _i32, _i32, _vp, _vp, _i32,
                              _f32, _vp, _vp, _i64, _vp]),
    "stc_conv_wgrad_workspace": (_i64, [_i32, _i32, _i32, _i32, _i32, _i32]),
    "stc_conv_wgrad_ex": (_i32, [_i32, _i32, _i32, View, _i32, _vp, _vp, _i32, _f32, View, _i32, _i32, _vp, _vp, _i32,
                                 _f32, _vp, _vp, _vp, _i64, _vp]),
    "stc_conv_wgrad_query": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp]),
    "stc_pack_weight": (_i32, [_i32, _i32, _vp, _i32, _i32, _vp, _i32, _i32, _vp]),
    "stc_pack_weights": (_i32, [_i32, _i32, _vp, _vp]),
    "stc_chan_stats": (_i32, [_i32, _i32, View, _i32, _vp, _i32, _vp]),
    "stc_chan_stats_chunks": (_i32, [_i32, _i32, _i32]),
    "stc_chan_sum": (_i32, [_i32, _i32, View, _i32, _i32, _vp, _i32, _vp, _vp]),
    "stc_bn_apply": (_i32, [_i32, _i32, View, _i32, _vp, _vp, View, _f32, View, _f32, _vp]),
    "stc_bn_finalize": (_i32, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _vp, _vp, _vp, _vp, _vp]),
    "stc_bn_bwd_reduce": (_i32, [_i32, _i32, View, _i32, _vp, _vp, _vp, _vp, View, _f32, View, _f32, _vp, _i32,
                                 _vp]),
    "stc_bn_bwd_apply": (_i32, [_i32, _i32, View, _i32, _vp, _vp, _vp, _vp, _vp, View, _f32, View, _f32, _vp, _i32,
                                View, _vp, _vp, _vp]),
    "stc_tanh_bias_bwd": (_i32, [_i32, _i32, _i32, _i32, _i32, _vp, _vp, View, _vp, _vp, _i32, _vp]),
    "stc_gather_nchw": (_i32, [_i32, _i32, _i32, _i32, _i32, _vp, _vp, View, _i32, _vp]),
    "stc_scatter_nchw": (_i32, [_i32, _i32, _i32, _i32, View, _i32, _vp, _vp, _vp]),
    "stc_loss_parts": (_i32, [_i64]),
    "stc_loss_fwd": (_i32, [_i32, _vp, _vp, _f32, _i64, _vp, _vp, _vp]),
    "stc_loss_bwd": (_i32, [_i32, _vp, _vp, _f32, _i64, _vp, _vp, _vp]),
    "stc_loss_multi_parts": (_i32, [_i32, _vp]),
    "stc_loss_multi_fwd": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp]),
    "stc_loss_multi_bwd": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "stc_adam_step": (_i32, [_vp, _i32, _i64, _f32, _f32, _f32, _f32, _i32, _vp]),
    "stc_adam_elems_per_block": (_i32, []),
    "stc_conv_wgrad_rows": (_i32, [_i32, _i32, View, _i32, _i32, View, _i32, _i32, _vp, _vp, _i64, _vp]),
    "stc_conv_wgrad_rows_workspace": (_i64, [_i32, _i32, _i32, _i32]),
    "stc_adam_pack_step": (_i32, [_vp, _i32, _i64, _f32, _f32, _f32, _f32, _i32, _vp]),
    "stc_adam_pack_step_dev": (_i32, [_vp, _i32, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _f32, _f32, _f32, _vp]),
    "stc_adam_coef_dev": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    "stc_adam_pack_apply": (_i32, [_vp, _i32, _i64, _f32, _i32, _vp, _f32, _f32, _f32, _vp]),
    "stc_grad_accumulate": (_i32, [_i32, _vp, _vp, _vp, _vp]),
    "stc_infer_output": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "stc_istd_errors_workspace": (_i64, [_i32, _i32, _i32]),
    "stc_istd_errors": (_i32, [_vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _i64, _vp]),
    "stc_istd_ssim": (_i32, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _i64, _vp]),
    "stc_image_resize_workspace": (_i64, [_i32, _i32, _i32]),
    "stc_image_resize_f64": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _i64, _vp]),
    "stc_istd_typed_workspace": (_i64, [_i32, _i32]),
    "stc_istd_errors_ex": (_i32, [_vp, _i32, _vp, _i32, _vp, _i32, _i32, _vp, _vp, _i64, _vp]),
    "stc_istd_ssim_ex": (_i32, [_vp, _i32, _vp, _i32, _i32, _i32, _vp, _vp, _i64, _vp]),
    "stc_prepare_batch": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp]),
    "stc_prepare_batch_f32": (_i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp]),
    "stc_resize_linear": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "stc_warp_affine": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp]),
    "stc_resize_area": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "stc_time_next_main_kernel": (_i32, [_vp, _vp]),
    "stc_stream_wait": (_i32, [_vp, _vp]),
    "stc_last_error": (ctypes.c_char_p, []),
    "stc_version": (_i32, []),
}

EXPORTED = tuple(_SIGS)

_lib = None


def lib():
    """Load the library once; raise loudly if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"stcgan_amd: HIP library not built ({LIB_PATH}); run __graft_entry__.build()")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().stc_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_device = torch._C._cuda_getDevice


def stream():
    """The current HIP stream of the current device (the raw accessor: torch.cuda.current_stream() costs
    ~8 us of Python per call, and the step makes a few hundred launches)."""
    return ctypes.c_void_p(_raw_stream(_cur_device()))


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise ValueError(f"unsupported dtype {dt}")


def nhwc_view(t, c0=0, H=None, W=None):
    """View of a contiguous NHWC tensor [B, Ha, Wa, C] (channel offset c0, logical H x W).
    The view keeps a reference to ``t`` so the memory cannot be recycled before the call."""
    assert t.dim() == 4 and t.is_contiguous()
    _, Ha, Wa, C = t.shape
    H = Ha if H is None else H
    W = Wa if W is None else W
    assert 0 <= H <= Ha and 0 <= W <= Wa and 0 <= c0 < C, "view outside the tensor"
    v = View(t.data_ptr(), H, W, Ha * Wa * C, Wa * C, C, c0, 1, 0)
    v._keep = t
    return v


def layout_key(v):
    """The layout of a view as the kernels' routing sees it (extent, strides, channel offset, 16-byte alignment)."""
    return (v.H, v.W, v.bs, v.rs, v.ps, v.co, v.cs, (v.p or 0) % 16)


def nchw_view(t):
    """View of a contiguous NCHW tensor [B, C, H, W]."""
    assert t.dim() == 4 and t.is_contiguous()
    _, C, H, W = t.shape
    v = View(t.data_ptr(), H, W, C * H * W, W, 1, 0, H * W, 0)
    v._keep = t
    return v
