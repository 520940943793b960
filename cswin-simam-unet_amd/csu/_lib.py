"""ctypes binding of libcsu_hip.so (C ABI declared in include/csu.h).

torch is imported first on purpose: it loads its bundled HIP runtime (soname libamdhip64.so.7),
and the dynamic loader then resolves our library's DT_NEEDED to that same runtime, so torch's
device pointers and streams are valid for our kernels.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

# CSU_LIB_PATH: load another build of the library (A/B experiments)
LIB_PATH = os.environ.get("CSU_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libcsu_hip.so")

c_int32, c_float, c_void_p, c_size_t = ctypes.c_int32, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t

CSU_F32, CSU_BF16 = 0, 1


class StripeBranch(ctypes.Structure):
    _fields_ = [("H_sp", c_int32), ("W_sp", c_int32), ("ch_off", c_int32), ("_pad", c_int32),
                ("lepe_w", c_void_p), ("lepe_b", c_void_p), ("lepe_dw", c_void_p), ("lepe_db", c_void_p)]


class StripeArgs(ctypes.Structure):
    _fields_ = [("B", c_int32), ("reso", c_int32), ("C", c_int32), ("heads", c_int32), ("head_dim", c_int32),
                ("nbranch", c_int32), ("scale", c_float), ("_pad", c_int32), ("br", StripeBranch * 2),
                ("drop_rng", c_void_p), ("drop_site", ctypes.c_uint32), ("drop_p", c_float)]


class LnParamItem(ctypes.Structure):
    """csu_ln_param_item (include/csu.h)."""
    _fields_ = [("workspace", c_void_p), ("dgamma", c_void_p), ("dbeta", c_void_p), ("rows", c_int32), ("C", c_int32),
                ("nblocks", c_int32), ("_pad", c_int32)]


class WslabItem(ctypes.Structure):
    """csu_wslab_item (include/csu.h)."""
    _fields_ = [("slab", c_void_p), ("dst", c_void_p), ("N", c_int32), ("K", c_int32), ("tn", c_int32), ("tk", c_int32),
                ("chunks", c_int32), ("_pad", c_int32)]


class WgradGroupItem(ctypes.Structure):
    """csu_wgrad_group_item (include/csu.h)."""
    _fields_ = [("dy", c_void_p), ("x", c_void_p), ("dw_db", c_void_p), ("slab", c_void_p), ("M", ctypes.c_int64),
                ("N", c_int32), ("K", c_int32)]


class LepeReduceItem(ctypes.Structure):
    """csu_lepe_reduce_item (include/csu.h)."""
    _fields_ = [("part", c_void_p), ("dw", c_void_p * 2), ("db", c_void_p * 2), ("nblk", c_int32), ("channels", c_int32),
                ("nbranch", c_int32), ("_pad", c_int32)]


class MlpDropout(ctypes.Structure):
    """csu_mlp_dropout (include/csu.h)."""
    _fields_ = [("rng", c_void_p), ("site_hidden", ctypes.c_uint32), ("site_out", ctypes.c_uint32), ("p", c_float),
                ("row_scale", c_void_p), ("rows_per_sample", ctypes.c_int64)]


class GemmDesc(ctypes.Structure):
    """csu_gemm_desc (include/csu.h)."""
    _fields_ = [("M", ctypes.c_int64), ("N", c_int32), ("K", c_int32), ("a", c_void_p), ("b", c_void_p),
                ("lda", c_int32), ("ldb", c_int32), ("b_trans", c_int32), ("a_gelu", c_int32), ("bias", c_void_p),
                ("gelu_aux", c_void_p), ("resid", c_void_p), ("out", c_void_p), ("gelu_out", c_void_p),
                ("ldc", c_int32), ("out_dtype", c_int32), ("cfg", c_int32), ("_pad", c_int32)]


class HeadFold(ctypes.Structure):
    _fields_ = [("O", c_int32), ("w_out", c_void_p), ("b_out", c_void_p), ("w_h", c_void_p), ("dw_out", c_void_p),
                ("db_out", c_void_p), ("dw_h", c_void_p)]


class ConvGeom(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("B", "H", "W", "C", "OH", "OW", "N", "KH", "KW", "stride", "pad")]


# name -> (restype, argtypes); mirrors include/csu.h
_SIGS = {
    "csu_last_error_string": (ctypes.c_char_p, []),
    "csu_build_info": (ctypes.c_char_p, []),
    "csu_event_create": (ctypes.c_int, [ctypes.POINTER(c_void_p)]),
    "csu_event_destroy": (ctypes.c_int, [c_void_p]),
    "csu_event_record_ext": (ctypes.c_int, [c_void_p, c_void_p]),
    "csu_event_elapsed_ms": (ctypes.c_int, [c_void_p, c_void_p, ctypes.POINTER(c_float)]),
    "csu_stripe_attn_fwd": (ctypes.c_int, [ctypes.POINTER(StripeArgs), ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "csu_stripe_attn_bwd_workspace": (c_size_t, [ctypes.POINTER(StripeArgs)]),
    "csu_stripe_attn_bwd": (ctypes.c_int, [ctypes.POINTER(StripeArgs), ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_layernorm_fwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_float, ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                         ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "csu_layernorm_bwd_workspace": (c_size_t, [ctypes.c_int, ctypes.c_int]),
    "csu_layernorm_bwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                         ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                         c_void_p]),
    "csu_layernorm_bwd_ex": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                            c_void_p, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_simam_workspace": (c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "csu_simam_fwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_float, ctypes.c_int, c_void_p, ctypes.c_int,
                                     c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_simam_bwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, ctypes.c_int,
                                     c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_simam_fwd_fork": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_float, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_simam_bwd_join": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, ctypes.c_int,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_carafe_fwd": (ctypes.c_int, [ctypes.c_int] * 6 + [c_void_p] * 5),
    "csu_carafe_bwd": (ctypes.c_int, [ctypes.c_int] * 6 + [c_void_p] * 6),
    "csu_carafe_head_fwd": (ctypes.c_int, [ctypes.c_int] * 6 + [c_void_p] * 7),
    "csu_carafe_head_bwd_workspace": (c_size_t, [ctypes.c_int] * 5),
    "csu_carafe_head_bwd": (ctypes.c_int, [ctypes.c_int] * 6 + [c_void_p] * 11 + [c_size_t, c_void_p]),
    "csu_carafe_head_bwd_fold": (ctypes.c_int, [ctypes.c_int] * 6 + [c_void_p] * 9 + [ctypes.POINTER(HeadFold), c_void_p,
                                                                                     c_size_t, c_void_p]),
    "csu_head_fold_fwd": (ctypes.c_int, [ctypes.c_int, ctypes.c_int] + [c_void_p] * 6),
    "csu_head_fwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "csu_head_bwd_workspace": (c_size_t, [ctypes.c_long, ctypes.c_int]),
    "csu_head_bwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int] + [c_void_p] * 7 + [c_size_t, c_void_p]),
    "csu_colsum_workspace": (c_size_t, [ctypes.c_long, ctypes.c_long, ctypes.c_int]),
    "csu_colsum": (ctypes.c_int, [ctypes.c_long, ctypes.c_long, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_size_t,
                                  c_void_p]),
    "csu_linear_wgrad_workspace": (c_size_t, [ctypes.c_long, ctypes.c_int, ctypes.c_int]),
    "csu_linear_wgrad": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_linear_wgrad_tuned_workspace": (c_size_t, [ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_int]),
    "csu_linear_wgrad_tuned": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              c_void_p]),
    "csu_gemm": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, c_void_p, ctypes.c_int, c_void_p, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int,
                                ctypes.c_int, c_void_p]),
    "csu_cast_bf16_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_long, c_void_p]),
    "csu_adamw_chunk_elems": (ctypes.c_long, []),
    "csu_adamw_step": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_long, c_void_p, c_float, c_float, c_float, c_float,
                                      c_float, c_void_p, c_float, c_void_p]),
    "csu_adam_l2_step": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_long, c_void_p, c_float, c_float, c_float, c_float,
                                      c_float, c_void_p, c_float, c_void_p]),
    "csu_gemm_ex": (ctypes.c_int, [ctypes.POINTER(GemmDesc), c_void_p]),
    "csu_mlp_fwd_ln": (ctypes.c_int, [ctypes.c_long, ctypes.c_int] + [c_void_p] * 8 + [c_void_p, c_void_p, c_float, c_void_p,
                                                                               c_void_p, c_void_p, c_void_p]),
    "csu_gemm_ws_supported": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "csu_gemm_ws": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, c_void_p, ctypes.c_int, c_void_p, c_void_p,
                                   c_void_p, ctypes.c_int, c_void_p, c_void_p]),
    "csu_gemm_ws_ln_supported": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int]),
    "csu_gemm_ws_ln": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, c_void_p, ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "csu_gemm_ws_lnbwd_supported": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int]),
    "csu_gemm_ws_lnbwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int] + [c_void_p] * 11),
    "csu_frag_layout_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_long, c_void_p]),
    "csu_frag8_layout_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_long, c_void_p]),
    "csu_gemm_ws_e4m3": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, c_void_p, ctypes.c_int, c_void_p,
                                        c_void_p, ctypes.c_int, c_void_p, c_void_p, ctypes.c_int, c_void_p, c_void_p]),
    "csu_gemm_ws_ln_e4m3": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, c_void_p, ctypes.c_int, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float, c_void_p,
                                           c_void_p, c_void_p, c_void_p]),
    "csu_gemm_f32_workspace": (c_size_t, [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_long]),
    "csu_gemm_f32": (ctypes.c_int, [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_long, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_quant_e4m3_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_long, c_void_p]),
    "csu_fp8_gemm": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int] + [c_void_p] * 7),
    "csu_layernorm_fwd_fp8": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_float, ctypes.c_int] + [c_void_p] * 8),
    "csu_layernorm_fwd_fp8_dq": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_float, ctypes.c_int] + [c_void_p] * 9),
    "csu_dequant_e4m3_rows": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "csu_e4m3_layout_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_long, c_void_p]),
    "csu_quant_e4m3_shadow_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_long, c_void_p]),
    "csu_mlp_fp8_supported": (ctypes.c_int, [ctypes.c_int]),
    "csu_mlp_fwd_ex": (ctypes.c_int, [ctypes.c_long, ctypes.c_int] + [c_void_p] * 7 + [ctypes.POINTER(MlpDropout), ctypes.c_int,
                                                                                       c_void_p]),
    "csu_mlp_bwd_ex": (ctypes.c_int, [ctypes.c_long, ctypes.c_int] + [c_void_p] * 8 + [ctypes.POINTER(MlpDropout), ctypes.c_int,
                                                                                       c_void_p]),
    "csu_mlp_fp8_fwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int] + [c_void_p] * 9 + [ctypes.POINTER(MlpDropout), c_void_p]),
    "csu_mlp_fp8_fwd_ln": (ctypes.c_int, [ctypes.c_long, ctypes.c_int] + [c_void_p] * 9 + [ctypes.POINTER(MlpDropout), c_void_p,
                                          c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "csu_mlp_fp8_bwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int] + [c_void_p] * 11 + [ctypes.POINTER(MlpDropout),
                                                                                         c_void_p]),
    "csu_mlp_supported": (ctypes.c_int, [ctypes.c_int]),
    "csu_dropout_apply": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, ctypes.c_int,
                                         c_void_p, c_void_p, ctypes.c_long, c_void_p, ctypes.c_uint, c_float, c_void_p]),
    "csu_dropout_mask": (ctypes.c_int, [ctypes.c_long, c_void_p, ctypes.c_uint, c_float, c_void_p, c_void_p]),
    "csu_rng_advance": (ctypes.c_int, [c_void_p, c_void_p, c_void_p]),
    "csu_droppath_scale": (ctypes.c_int, [ctypes.c_long, c_void_p, ctypes.c_uint, c_float, c_void_p, c_void_p]),
    "csu_layernorm_param_reduce": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "csu_layernorm_param_reduce_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, c_void_p]),
    "csu_linear_wgrad_deferred": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                                 c_void_p, c_size_t, ctypes.POINTER(WslabItem), c_void_p]),
    "csu_wslab_reduce_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, c_void_p]),
    "csu_stripe_attn_bwd_ex": (ctypes.c_int, [ctypes.POINTER(StripeArgs), ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, ctypes.c_int, c_void_p]),
    "csu_stripe_lepe_nblk": (ctypes.c_int, [ctypes.POINTER(StripeArgs), ctypes.c_int]),
    "csu_stripe_lepe_reduce_batch": (ctypes.c_int, [c_void_p, ctypes.c_int, c_void_p]),
    "csu_linear_wgrad_group_plan": (c_size_t, [ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "csu_linear_wgrad_group": (ctypes.c_int, [c_void_p, ctypes.c_int, c_void_p]),
    "csu_augment_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p]),
    "csu_bn_workspace": (c_size_t, [ctypes.c_long, ctypes.c_int]),
    "csu_bn_relu_fwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_float, c_float, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p,
                                       c_void_p, c_size_t, c_void_p]),
    "csu_bn_relu_bwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_size_t, c_void_p]),
    "csu_maxpool2_fwd": (ctypes.c_int, [ctypes.c_int] * 5 + [c_void_p, c_void_p, c_void_p]),
    "csu_maxpool2_bwd": (ctypes.c_int, [ctypes.c_int] * 5 + [c_void_p, ctypes.c_int, c_void_p, c_void_p, c_void_p]),
    "csu_grad_join": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, c_void_p, ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
    "csu_bce_loss_workspace": (c_size_t, [ctypes.c_long]),
    "csu_bce_loss_fwd": (ctypes.c_int, [ctypes.c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_bce_loss_fwd_stats": (ctypes.c_int, [ctypes.c_long] + [c_void_p] * 5 + [c_size_t, c_void_p]),
    "csu_bce_loss_bwd": (ctypes.c_int, [ctypes.c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "csu_pack_nhwc_bf16": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p,
                                          c_void_p, c_void_p]),
    "csu_stripe_lepe_wgrad": (ctypes.c_int, [ctypes.POINTER(StripeArgs), ctypes.c_int, c_void_p, c_void_p, c_void_p, c_size_t,
                                             c_void_p]),
    "csu_mlp_fwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "csu_mlp_fwd_dp": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, ctypes.POINTER(MlpDropout), c_void_p]),
    "csu_mlp_bwd_dp": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, ctypes.POINTER(MlpDropout), c_void_p]),
    "csu_mlp_bwd": (ctypes.c_int, [ctypes.c_long, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p]),
    "csu_conv2d_fwd": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p]),
    "csu_conv2d_dgrad": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "csu_conv2d_ex": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p, ctypes.c_int, c_void_p]),
    "csu_conv2d_workspace": (c_size_t, [ctypes.c_int, ctypes.POINTER(ConvGeom), ctypes.c_int]),
    "csu_conv2d_fwd_ws": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int] + [c_void_p] * 5 + [c_size_t, c_void_p]),
    "csu_conv2d_dgrad_ws": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int] + [c_void_p] * 5 + [c_size_t, c_void_p]),
    "csu_conv2d_wgrad_workspace": (c_size_t, [ctypes.POINTER(ConvGeom)]),
    "csu_conv2d_wgrad_workspace_ex": (c_size_t, [ctypes.POINTER(ConvGeom), ctypes.c_int]),
    "csu_conv2d_split_ok": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int]),
    "csu_conv2d_fwd_split": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, ctypes.c_int, c_void_p,
                                            c_void_p, c_void_p, c_void_p]),
    "csu_conv2d_dgrad_split": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                              ctypes.c_int, c_void_p]),
    "csu_conv2d_wgrad_split_oihw": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, ctypes.c_int,
                                                   c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "csu_conv2d_wgrad_ex": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, ctypes.c_int,
                                           c_void_p, c_void_p, c_size_t, ctypes.c_int, c_void_p]),
    "csu_conv2d_wgrad": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_size_t, c_void_p]),
    "csu_conv2d_wgrad_oihw": (ctypes.c_int, [ctypes.POINTER(ConvGeom), ctypes.c_int, c_void_p, c_void_p, ctypes.c_int,
                                             c_void_p, c_void_p, c_size_t, c_void_p]),
}

_lib = None
_lock = threading.Lock()


class CsuError(RuntimeError):
    pass


def lib():
    """The loaded library; raises loudly when it has not been built (no fallback exists)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise CsuError(f"libcsu_hip.so not built ({LIB_PATH}); run `python __graft_entry__.py build` "
                                   "or `make -C cswin-simam-unet_amd/csrc`")
                L = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in _SIGS.items():
                    fn = getattr(L, name)
                    fn.restype, fn.argtypes = res, args
                _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().csu_last_error_string().decode(errors="replace")
        raise CsuError(f"{what} failed (code {rc}): {msg}")


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return CSU_F32
    if t.dtype == torch.bfloat16:
        return CSU_BF16
    raise CsuError(f"unsupported dtype {t.dtype} (float32 or bfloat16)")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(*ts: torch.Tensor):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise CsuError("csu kernels run on the MI355X only: got a CPU tensor (there is no CPU fallback)")
