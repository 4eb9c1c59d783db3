"""ctypes binding of libskeldiff.so (the C ABI declared in include/skeldiff.h).

The library is built in-tree by `skeletondiffusion_amd.build.build_library()` (hipcc,
--offload-arch=gfx950).  There is no fallback: if the library is missing or cannot be loaded,
every sampling entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
# SKELDIFF_LIB: load another build of the library (e.g. the libskeldiff_dbg.so diagnostic variant)
LIB_PATH = os.environ.get("SKELDIFF_LIB") or os.path.join(HERE, "libskeldiff.so")

# include/skeldiff.h SD_ABI_VERSION: a library of another ABI is refused at load (round 4 changed
# signatures under the same number; a client built against the old header would pass shifted
# arguments instead of failing cleanly)
SD_ABI_VERSION = 4

SD_FLAG_GRAPH = 1
SD_FLAG_DEVICE_START = 2
SD_FLAG_DEVICE_NOISE = 4
SD_FLAG_NO_CLIP = 8

# every symbol include/skeldiff.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "sd_abi_version", "sd_last_error", "sd_build_info", "sd_plan_create", "sd_plan_destroy", "sd_plan_num_tensors",
    "sd_plan_tensor_name", "sd_plan_tensor_numel", "sd_plan_dims", "sd_plan_set_tensor", "sd_plan_finalize",
    "sd_workspace_bytes", "sd_denoiser_forward", "sd_p_sample_update", "sd_sample_loop",
    "sd_noise_fill", "sd_philox_raw", "sd_plan_kernels_per_step", "sd_plan_step_flops", "sd_profile_step",
    "sd_test_graph_linear", "sd_test_attention", "sd_test_set_kernel_variant", "sd_test_qkv_attention",
    "sd_test_graph_linear_layout", "sd_pairwise_distances", "sd_ade_fde",
    "sd_plan_set_precision", "sd_mm_ade_fde", "sd_gru_decode_workspace_bytes", "sd_gru_decode",
    "sd_gru_encode_workspace_bytes", "sd_gru_encode", "sd_gl_train_workspace_bytes", "sd_gl_train_forward",
    "sd_gl_train_backward", "sd_plan_set_option", "sd_plan_get_option", "sd_denoiser_trace",
    "sd_workspace_status", "sd_attn_train_forward",
    "sd_attn_train_backward", "sd_film_tanh_forward", "sd_film_tanh_backward", "sd_l1norm_rows_forward",
    "sd_l1norm_rows_backward", "sd_rmsnorm_workspace_bytes", "sd_rmsnorm_forward", "sd_rmsnorm_backward",
    "sd_mahalanobis_loss_forward", "sd_mahalanobis_loss_backward", "sd_best_of_k", "sd_best_of_k_backward",
    "sd_pose_loss", "sd_test_set_split_route",
)

# sd_plan_set_option keys (include/skeldiff.h)
(SD_OPT_KERNEL_VARIANT, SD_OPT_GL4_TILE, SD_OPT_ROW_CHAINS, SD_OPT_PRECISION, SD_OPT_GL4_STAGING,
 SD_OPT_SPLIT_ROUTE, SD_OPT_LAST_CHAINS, SD_OPT_LAST_ROUTE, SD_OPT_UPDATE_KERNEL, SD_OPT_V5_MIX,
 SD_OPT_ATTENTION) = range(1, 12)
# SD_OPT_LAST_ROUTE bits (sd::RouteBits)
ROUTE_BITS = {1: "k_gl4 one-kernel", 2: "k_gl4 fused to_qkv+attention", 4: "k_gl4y GEMM phase",
              8: "k_gl4t GEMM phase", 16: "k_gl4 MODE 2/3 mixing phase", 32: "v5 k_gl5 mixing", 64: "exact-f32 kernels",
              128: "k_attention", 1024: "k_attention_mix (to_qkv mixing inside the attention kernel)"}
SD_STATUS_F16_RANGE = 1


class SDPlanDesc(ctypes.Structure):
    _fields_ = [
        ("num_nodes", ctypes.c_int32),
        ("latent_dim", ctypes.c_int32),
        ("cond_dim", ctypes.c_int32),
        ("out_dim", ctypes.c_int32),
        ("depth", ctypes.c_int32),
        ("attn_heads", ctypes.c_int32),
        ("attn_dim_head", ctypes.c_int32),
        ("use_attention", ctypes.c_int32),
        ("self_condition", ctypes.c_int32),
        ("learn_influence", ctypes.c_int32),
        ("num_node_types", ctypes.c_int32),
        ("node_types", ctypes.POINTER(ctypes.c_int64)),
        ("timesteps", ctypes.c_int32),
        ("isotropic", ctypes.c_int32),
        ("activation", ctypes.c_int32),
        ("sinusoidal_theta", ctypes.c_float),
        ("objective", ctypes.c_int32),
        ("norm_type", ctypes.c_int32),  # ABI 4: 0 'none', 1 'layer'
    ]


class SDGruDecoderDesc(ctypes.Structure):
    """mirrors struct sd_gru_decoder_desc (include/skeldiff.h)"""
    _fields_ = [(n, ctypes.c_int32) for n in ("num_nodes", "feature_size", "latent_size", "hidden_size",
                                              "num_node_types")] + \
               [("node_types", ctypes.POINTER(ctypes.c_int64))] + \
               [(n, ctypes.c_void_p) for n in ("init_G", "init_weight", "init_bias", "G", "G_add", "weight_ih",
                                               "weight_hh", "bias_ih", "bias_hh", "fc_G", "fc_weight", "fc_bias")]


class SkelDiffError(RuntimeError):
    pass


_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


def _declare(lib: ctypes.CDLL) -> None:
    vp, i32, i64, u64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_size_t
    sig = {
        "sd_abi_version": (i32, []),
        "sd_last_error": (ctypes.c_char_p, []),
        "sd_build_info": (ctypes.c_char_p, []),
        "sd_plan_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(SDPlanDesc)]),
        "sd_plan_destroy": (None, [vp]),
        "sd_plan_num_tensors": (i32, [vp]),
        "sd_plan_tensor_name": (ctypes.c_char_p, [vp, i32]),
        "sd_plan_tensor_numel": (i64, [vp, i32]),
        "sd_plan_set_tensor": (ctypes.c_int, [vp, ctypes.c_char_p, vp, i64, vp]),
        "sd_plan_finalize": (ctypes.c_int, [vp, vp]),
        "sd_workspace_bytes": (sz, [vp, i64]),
        "sd_plan_dims": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int32)]),
        "sd_denoiser_forward": (ctypes.c_int, [vp, vp, vp, i64, i32, vp, i64, vp, sz, vp]),
        "sd_workspace_status": (ctypes.c_int, [vp, vp, sz, ctypes.POINTER(ctypes.c_uint32), vp]),
        "sd_denoiser_trace": (ctypes.c_int, [vp, vp, vp, i64, i32, vp, i64, vp, sz, ctypes.POINTER(vp), i32, vp]),
        "sd_p_sample_update": (ctypes.c_int, [vp, vp, vp, vp, i64, u64, i64, i32, vp, vp, i64, vp, i64, i64, i32, vp]),
        "sd_sample_loop": (ctypes.c_int, [vp, vp, vp, i64, vp, u64, i64, vp, vp, vp, vp, vp, i64, vp, sz, i32, vp]),
        "sd_noise_fill": (ctypes.c_int, [vp, i64, i64, u64, i64, i32, vp]),
        "sd_philox_raw": (ctypes.c_int, [vp, i64, i64, u64, i64, i32, vp]),
        "sd_plan_kernels_per_step": (i32, [vp]),
        "sd_plan_step_flops": (ctypes.c_int, [vp, i64, ctypes.POINTER(ctypes.c_double)]),
        "sd_test_graph_linear": (ctypes.c_int, [vp, i32, i64, vp, i32, vp, vp, ctypes.POINTER(ctypes.c_int64), vp,
                                                vp, i32, vp, vp, i64, i32, i32, i32, vp]),
        "sd_test_attention": (ctypes.c_int, [vp, vp, i64, i32, i32, i32, vp]),
        "sd_test_set_kernel_variant": (ctypes.c_int, [i32, i32]),
        "sd_test_set_split_route": (ctypes.c_int, [i32]),
        "sd_plan_set_precision": (ctypes.c_int, [vp, i32]),
        "sd_plan_set_option": (ctypes.c_int, [vp, i32, i64]),
        "sd_plan_get_option": (ctypes.c_int, [vp, i32, ctypes.POINTER(ctypes.c_int64)]),
        "sd_mm_ade_fde": (ctypes.c_int, [vp, vp, vp, i64, vp, i64, i32, i32, i64, vp, vp, vp, vp, vp]),
        "sd_gru_decode_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(SDGruDecoderDesc), i64, i32]),
        "sd_gru_decode": (ctypes.c_int, [ctypes.POINTER(SDGruDecoderDesc), vp, vp, i64, i32, vp, vp,
                                         ctypes.c_size_t, vp]),
        "sd_gru_encode_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(SDGruDecoderDesc), i64, i32]),
        "sd_gru_encode": (ctypes.c_int, [ctypes.POINTER(SDGruDecoderDesc), vp, i64, i32, vp, vp, ctypes.c_size_t, vp]),
        "sd_pairwise_distances": (ctypes.c_int, [vp, i64, i32, i64, vp, vp, vp]),
        "sd_ade_fde": (ctypes.c_int, [vp, vp, i64, i32, i32, i64, vp, vp, vp, vp, vp]),
        "sd_test_qkv_attention": (ctypes.c_int, [vp, i32, vp, ctypes.POINTER(ctypes.c_int64), vp, vp, i64, i32, i32,
                                                 i32, i32, vp]),
        "sd_test_graph_linear_layout": (ctypes.c_int, [vp, i32, i64, vp, i32, vp, vp, ctypes.POINTER(ctypes.c_int64),
                                                       vp, vp, i32, vp, vp, i64, i32, i32, i32, i32, vp]),
        "sd_gl_train_workspace_bytes": (sz, [i64, i32, i32, i32, i32]),
        "sd_gl_train_forward": (ctypes.c_int, [vp, vp, vp, vp, i32, vp, i64, i32, i32, i32, vp, vp, vp]),
        "sd_gl_train_backward": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, vp, i64, i32, i32, i32, vp, vp, vp, vp, vp,
                                                sz, vp]),
        "sd_attn_train_forward": (ctypes.c_int, [vp, vp, i64, i32, i32, i32, ctypes.c_float, vp]),
        "sd_attn_train_backward": (ctypes.c_int, [vp, vp, vp, i64, i32, i32, i32, ctypes.c_float, vp]),
        "sd_film_tanh_forward": (ctypes.c_int, [vp, vp, vp, i64, i32, i32, vp]),
        "sd_film_tanh_backward": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i32, i32, vp]),
        "sd_l1norm_rows_forward": (ctypes.c_int, [vp, vp, i32, i32, ctypes.c_float, vp]),
        "sd_l1norm_rows_backward": (ctypes.c_int, [vp, vp, vp, i32, i32, ctypes.c_float, vp]),
        "sd_rmsnorm_workspace_bytes": (sz, [i64, i32]),
        "sd_rmsnorm_forward": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, ctypes.c_float, ctypes.c_float, vp]),
        "sd_rmsnorm_backward": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i32, ctypes.c_float, ctypes.c_float, vp,
                                               sz, vp]),
        "sd_mahalanobis_loss_forward": (ctypes.c_int, [vp, vp, vp, vp, i32, i64, i32, i32, i32, i32, vp, vp]),
        "sd_mahalanobis_loss_backward": (ctypes.c_int, [vp, vp, vp, vp, i32, vp, i64, i32, i32, i32, i32, vp, vp]),
        "sd_best_of_k": (ctypes.c_int, [vp, vp, i64, i32, vp, vp, vp]),
        "sd_best_of_k_backward": (ctypes.c_int, [vp, vp, i64, i32, vp, vp]),
        "sd_pose_loss": (ctypes.c_int, [vp, vp, i64, i32, i32, i32, i32, i32, vp, vp]),
        "sd_profile_step": (ctypes.c_int, [vp, vp, vp, i64, i32, i64, vp, sz, i32, ctypes.POINTER(ctypes.c_float),
                                           ctypes.POINTER(ctypes.c_int32), vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib() -> ctypes.CDLL:
    """Load libskeldiff.so (once).  Raises SkelDiffError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise SkelDiffError(
                    f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                    "(hipcc --offload-arch=gfx950).  There is no CPU fallback for sampling.")
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            _declare(handle)
            abi = handle.sd_abi_version()
            if abi != SD_ABI_VERSION:
                raise SkelDiffError(f"{LIB_PATH} has ABI version {abi}, this binding needs {SD_ABI_VERSION}: "
                                    "rebuild it with skeletondiffusion_amd.build.build_library()")
            info = handle.sd_build_info().decode()
            # the product library is built without packed-FP32 instructions; a
            # diagnostic build is loaded only when named explicitly through SKELDIFF_LIB
            if info != "no-packed-fp32" and not os.environ.get("SKELDIFF_LIB"):
                raise SkelDiffError(f"{LIB_PATH} was built as {info!r}, not the product build "
                                    "(no-packed-fp32): rebuild it with skeletondiffusion_amd.build.build_library()")
            _lib = handle
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().sd_last_error()
        raise SkelDiffError(f"libskeldiff error {rc}: {msg.decode() if msg else '?'}")


def ptr(t) -> Optional[int]:
    """data_ptr of a torch tensor (None for None)."""
    return None if t is None else t.data_ptr()
