"""ctypes binding of libvspike.so — the C-ABI declared in include/vspike.h.

The library is the ONLY compute path: there is no CPU or torch fallback.  If it is missing, or
no GPU is visible, the ops raise.  Tensors cross the boundary as raw device pointers + sizes;
kernels are enqueued on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os

import torch

from .build import LIB_PATH

VS_F32, VS_BF16, VS_U8, VS_FP8 = 0, 1, 2, 3
EPI_BIAS, EPI_GELU, EPI_RELU, EPI_RESIDUAL, EPI_POS = 0x1, 0x2, 0x4, 0x8, 0x10
EPI_GELU_BWD, EPI_RELU_BWD, EPI_ATOMIC, EPI_ACCUM = 0x20, 0x40, 0x80, 0x100
EPI_GELU_GRAD, EPI_MUL_AUX = 0x200, 0x400
BWD_DEFER_JOIN = 0x1
BWD_DEFER_LAST = 0x2
BWD_FUSE_LN = 0x4
TIMER_ATTN_FWD, TIMER_ATTN_BWD, TIMER_GEMM, TIMER_GEMM_DW, TIMER_LN_FWD, TIMER_LN_BWD, TIMER_ADAMW, TIMER_MISC = range(8)
TIMER_NAMES = ("attn_fwd", "attn_bwd", "gemm", "gemm_dw", "ln_fwd", "ln_bwd", "adamw", "misc",
               # the block executor's products (vspike.h VS_TIMER_FWD_QKV ..): fwd, dX, dW of each Linear
               "fwd_qkv", "fwd_proj", "fwd_fc1", "fwd_fc2", "dx_fc2", "dx_fc1", "dx_proj", "dx_qkv",
               "dw_fc2", "dw_fc1", "dw_proj", "dw_qkv",
               # the fused MLP (a_pre == NULL in vs_vit_layer): forward, backward GELU' product
               "fwd_mlp", "dx_mlp",
               # the MX-FP8 forward's operand quantisation (compute_dtype fp8)
               "fp8_quant",
               # the R3D-18 encoder (BASELINE C4): conv forward / dX / dW (flops), BatchNorm + helpers (bytes)
               "conv_fwd", "conv_dx", "conv_dw", "bn")

# vspike.h VS_PATH_* (dispatch counters) and VS_KNOB_* (A/B and test knobs), in id order
PATH_NAMES = ("gemm_dw", "gemm_skinny", "gemm_slab", "gemm_big", "gemm_wres", "gemm_wslab", "gemm_panel",
              "gemm_fullk", "gemm_ring", "gemm_tile", "gemm_f32", "gemm_ln_fwd", "gemm_ln_bwd", "attn_fwd",
              "attn_bwd", "attn_f32", "patch_fused", "dw_grouped", "mlp_fwd", "mlp_bwd", "gemm_fp8", "patch_dw",
              "conv_igemm", "conv_dw", "gemm_g256", "gemm_dw256")
PATH_COUNT = 26
KNOB_NAMES = ("dw_old", "no_skinny", "no_slab", "no_big", "no_wres", "wres_gbwd", "no_wslab", "wslab", "wslab_g",
              "panel", "no_panel", "panel_grid", "no_fullk", "no_ring", "no_lnf_fuse", "no_ln_fuse", "dw_bm", "dw_bn",
              "dw_splits", "dw_stages", "ln_blocks", "dh_f32", "no_patch_fused", "no_dw_group", "attn_variant", "slab_wv", "wres_wv", "wres_dbg",
              "g256", "g256_grid", "g256_dbg", "no_dw256", "g256_stagger", "conv_dw128", "conv_mfma", "g256_a3", "dw256_all", "ln_fwd_blocks")
KNOB_COUNT = 40

c_i32, c_i64, c_u32, c_f32, c_p, c_sz = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_float,
                                         ctypes.c_void_p, ctypes.c_size_t)


class VsError(RuntimeError):
    pass


class GemmDesc(ctypes.Structure):
    _fields_ = [("dtype", c_i32), ("out_dtype", c_i32), ("a_kcontig", c_i32), ("b_kcontig", c_i32),
                ("M", c_i64), ("N", c_i64), ("K", c_i64),
                ("a", c_p), ("lda", c_i64), ("b", c_p), ("ldb", c_i64), ("c", c_p), ("ldc", c_i64),
                ("epilogue", c_u32), ("alpha", c_f32), ("bias", c_p),
                ("residual", c_p), ("ld_residual", c_i64), ("pos", c_p), ("pos_rows", c_i64),
                ("aux_in", c_p), ("ld_aux_in", c_i64), ("aux_out", c_p), ("ld_aux_out", c_i64),
                ("split_k", c_i32), ("reserved", c_i32), ("a_rowsum", c_p), ("workspace", c_p),
                ("workspace_bytes", c_i64)]


class Conv3dDesc(ctypes.Structure):
    _fields_ = [("N", c_i64), ("Di", c_i64), ("Hi", c_i64), ("Wi", c_i64), ("Ci", c_i64),
                ("Do", c_i64), ("Ho", c_i64), ("Wo", c_i64), ("Co", c_i64),
                ("kd", c_i32), ("kh", c_i32), ("kw", c_i32), ("sd", c_i32), ("sh", c_i32), ("sw", c_i32),
                ("pd", c_i32), ("ph", c_i32), ("pw", c_i32), ("reserved", c_i32)]


class VitLayer(ctypes.Structure):
    _fields_ = [("dtype", c_i32), ("heads", c_i32), ("batch", c_i64), ("tokens", c_i64), ("hidden", c_i64),
                ("mlp", c_i64), ("ln_eps", c_f32), ("attn_scale", c_f32),
                ("ln1_g", c_p), ("ln1_b", c_p), ("ln2_g", c_p), ("ln2_b", c_p),
                ("w_qkv", c_p), ("b_qkv", c_p), ("w_proj", c_p), ("b_proj", c_p),
                ("w_fc1", c_p), ("b_fc1", c_p), ("w_fc2", c_p), ("b_fc2", c_p),
                ("x_in", c_p), ("h1", c_p), ("mean1", c_p), ("rstd1", c_p), ("qkv", c_p), ("attn_o", c_p),
                ("lse", c_p), ("y", c_p), ("h2", c_p), ("mean2", c_p), ("rstd2", c_p), ("a_pre", c_p),
                ("a_act", c_p), ("x_out", c_p), ("fp8_ws", c_p), ("fp8_ws_bytes", c_i64),
                ("next_ln_g", c_p), ("next_ln_b", c_p), ("next_h1", c_p), ("next_mean1", c_p), ("next_rstd1", c_p),
                ("ln1_ready", c_i32), ("reserved7", c_i32)]


class VitLayerGrad(ctypes.Structure):
    _fields_ = [("ln1_g", c_p), ("ln1_b", c_p), ("ln2_g", c_p), ("ln2_b", c_p),
                ("w_qkv", c_p), ("b_qkv", c_p), ("w_proj", c_p), ("b_proj", c_p),
                ("w_fc1", c_p), ("b_fc1", c_p), ("w_fc2", c_p), ("b_fc2", c_p),
                ("dx_out", c_p), ("dx_out_lp", c_p), ("dx_in", c_p), ("dx_in_lp", c_p),
                ("d_a", c_p), ("d_h", c_p), ("dy", c_p), ("dy_lp", c_p), ("d_o", c_p), ("d_qkv", c_p),
                ("attn_ws", c_p), ("ln_ws", c_p), ("gemm_ws", c_p), ("gemm_ws_bytes", c_i64),
                ("flags", c_i32), ("reserved", c_i32), ("chain", c_p)]


# every entry point of include/vspike.h: name -> (restype, argtypes)
PROTOTYPES = {
    "vs_version": (ctypes.c_int, []),
    "vs_build_id": (ctypes.c_char_p, []),
    "vs_dispatch_counts": (ctypes.c_int, [ctypes.POINTER(c_i64), ctypes.c_int]),
    "vs_dispatch_reset": (ctypes.c_int, []),
    "vs_g256_scratch_free": (ctypes.c_int, []),
    "vs_knob_get": (ctypes.c_int, [ctypes.c_int]),
    "vs_knob_set": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "vs_knob_default": (ctypes.c_int, [ctypes.c_int]),
    "vs_debug_knobs": (ctypes.c_int, []),
    "vs_mse_loss": (ctypes.c_int, [c_i64, c_p, c_p, c_p, c_p, c_f32, c_p, c_p]),
    "vs_comm_unique_id": (ctypes.c_int, [c_p]),
    "vs_comm_init": (ctypes.c_int, [ctypes.POINTER(c_p), c_p, c_i32, c_i32]),
    "vs_comm_allreduce_bucket": (ctypes.c_int, [c_p, c_p, c_i64, c_i32, c_p]),
    "vs_comm_finalize": (ctypes.c_int, [c_p]),
    "vs_mse_loss_bwd": (ctypes.c_int, [c_i64, c_p, c_p, c_p, c_p, c_p]),
    "vs_last_error": (ctypes.c_char_p, []),
    "vs_device_arch": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "vs_struct_size": (ctypes.c_int, [ctypes.c_int]),
    "vs_gemm": (ctypes.c_int, [ctypes.POINTER(GemmDesc), c_p]),
    "vs_layernorm_fwd": (ctypes.c_int, [c_i32, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_f32, c_p, c_i64, c_p, c_p,
                                        c_p]),
    "vs_layernorm_bwd_workspace_bytes": (c_sz, [c_i64, c_i64]),
    "vs_gemm_splitk_workspace_bytes": (c_sz, [c_i32, c_i64, c_i64, c_i64]),
    "vs_video_preprocess": (ctypes.c_int, [c_i32, c_i64, c_i64, c_i64, c_i64, c_p, ctypes.POINTER(c_i32), c_i32,
                                           c_i64, ctypes.POINTER(c_f32), ctypes.POINTER(c_f32), c_p, c_p]),
    "vs_layernorm_bwd": (ctypes.c_int, [c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p,
                                        c_i64, c_p, c_p, c_p, c_p, c_p]),
    "vs_layernorm_bwd_dt": (ctypes.c_int, [ctypes.c_int32, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p,
                                        c_i64, c_p, c_p, c_p, c_p, c_p]),
    "vs_gemm_ln_fwd": (ctypes.c_int, [ctypes.POINTER(GemmDesc), c_p, c_p, ctypes.c_float, c_p, c_i64, c_p, c_p, c_p]),
    "vs_gemm_ln_bwd": (ctypes.c_int, [ctypes.POINTER(GemmDesc), c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64,
                                      c_p, c_p, c_p, c_p, c_p]),
    "vs_mlp_fused_ok": (ctypes.c_int, [c_i64, c_i64, c_i64]),
    "vs_mlp_fwd_ln": (ctypes.c_int, [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64,
                                     c_p, c_p, c_f32, c_p, c_i64, c_p, c_p, c_p]),
    "vs_quant_mxfp8": (ctypes.c_int, [c_i32, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p]),
    "vs_gemm_mxfp8": (ctypes.c_int, [ctypes.POINTER(GemmDesc), c_p, c_i64, c_p, c_i64, c_p]),
    "vs_mlp_fwd": (ctypes.c_int, [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p]),
    "vs_mlp_bwd_da": (ctypes.c_int, [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p, c_i64, c_p,
                                     c_i64, c_p]),
    "vs_attn_fwd": (ctypes.c_int, [c_i32, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_f32, c_p]),
    "vs_attn_bwd_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64, c_i64]),
    "vs_attn_redo_count": (ctypes.c_int, [ctypes.POINTER(c_i64), c_i32]),
    "vs_attn_bwd": (ctypes.c_int, [c_i32, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p,
                                   c_p, c_i64, c_p, c_f32, c_p]),
    "vs_patch_im2col": (ctypes.c_int, [c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "vs_sinusoid_table": (ctypes.c_int, [c_i64, c_i64, c_p, c_p]),
    "vs_patch_embed_fwd": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64,
                                          c_p, c_p, c_p]),
    "vs_patch_embed_dw_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "vs_patch_embed_dw": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_i64, c_i64, c_p,
                                         c_i64, c_p, c_p, c_i64, c_p]),
    "vs_colsum": (ctypes.c_int, [c_i32, c_i64, c_i64, c_p, c_i64, c_p, c_p]),
    "vs_cast": (ctypes.c_int, [c_i32, c_i32, c_i64, c_p, c_p, c_p]),
    "vs_poisson_workspace_bytes": (c_sz, [c_i64]),
    "vs_poisson_nll": (ctypes.c_int, [c_i64, c_p, c_p, c_p, c_p, c_f32, c_p, c_p]),
    "vs_poisson_nll_bwd": (ctypes.c_int, [c_i64, c_p, c_p, c_p, c_p, c_p]),
    "vs_adamw": (ctypes.c_int, [c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "vs_spike_metrics_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "vs_spike_metrics": (ctypes.c_int, [c_i64, c_i64, c_i64, c_p, c_p, c_i32, c_i64, c_i32, c_p, c_p, c_p, c_p,
                                        c_p]),
    "vs_shard_write": (ctypes.c_int, [ctypes.c_char_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p,
                                      ctypes.c_char_p]),
    "vs_shard_open": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.POINTER(c_i64)]),
    "vs_shard_key": (ctypes.c_int, [ctypes.c_void_p, c_i64, ctypes.c_char_p, c_i32]),
    "vs_shard_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(c_i64), c_i64, c_p, c_p, c_i32]),
    "vs_shard_close": (None, [ctypes.c_void_p]),
    "vs_shard_last_error": (ctypes.c_char_p, []),
    "vs_vit_layer_fwd": (ctypes.c_int, [ctypes.POINTER(VitLayer), c_p]),
    "vs_vit_fp8_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "vs_vit_layer_bwd": (ctypes.c_int, [ctypes.POINTER(VitLayer), ctypes.POINTER(VitLayerGrad), c_p]),
    "vs_bwd_chain_create": (ctypes.c_int, [ctypes.POINTER(c_p)]),
    "vs_bwd_chain_destroy": (ctypes.c_int, [c_p]),
    "vs_conv3d_fwd": (ctypes.c_int, [ctypes.POINTER(Conv3dDesc), c_p, c_p, c_p, c_p, c_p]),
    "vs_conv3d_stats_rows": (c_sz, [ctypes.POINTER(Conv3dDesc)]),
    "vs_conv3d_dx_workspace_bytes": (c_sz, [ctypes.POINTER(Conv3dDesc)]),
    "vs_conv3d_dx": (ctypes.c_int, [ctypes.POINTER(Conv3dDesc), c_p, c_p, c_p, c_i32, c_p, c_i64, c_p]),
    "vs_conv3d_dw_workspace_bytes": (c_sz, [ctypes.POINTER(Conv3dDesc)]),
    "vs_conv3d_dw": (ctypes.c_int, [ctypes.POINTER(Conv3dDesc), c_p, c_p, c_p, c_i32, c_p, c_i64, c_p]),
    "vs_bn3d_stats_workspace_bytes": (c_sz, [c_i64, c_i64]),
    "vs_bn3d_stats": (ctypes.c_int, [c_i64, c_i64, c_p, c_i64, c_p, c_p, c_f32, c_f32, c_p, c_p, c_p, c_p, c_p, c_p,
                                     c_p, c_p]),
    "vs_bn3d_apply": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_p, c_p, c_i32, c_p, c_p]),
    "vs_bn3d_bwd_workspace_bytes": (c_sz, [c_i64, c_i64]),
    "vs_bn3d_bwd": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "vs_bn3d_bwd_eval": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "vs_to_channels_last": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "vs_avgpool3d": (ctypes.c_int, [c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "vs_avgpool3d_bwd": (ctypes.c_int, [c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "vs_timing_enable": (ctypes.c_int, [ctypes.c_int]),
    "vs_timing_collect": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(c_i64), ctypes.POINTER(ctypes.c_double)]),
    "vs_timing_bytes": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
}

_LIB = None


def lib() -> ctypes.CDLL:
    """Load libvspike.so (built in-tree by vspike.build / __graft_entry__.build())."""
    global _LIB
    if _LIB is None:
        path = os.environ.get("VSPIKE_LIB") or LIB_PATH   # override: A/B timing of two builds
        if not os.path.exists(path):
            raise VsError(f"libvspike.so not found at {path}: build it with `python -m vspike.build` "
                          "(or __graft_entry__.build()); there is no fallback path")
        handle = ctypes.CDLL(path)
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        for which, st in enumerate((GemmDesc, VitLayer, VitLayerGrad, Conv3dDesc)):
            got = handle.vs_struct_size(which)
            if got != ctypes.sizeof(st):
                raise VsError(f"ABI mismatch: {st.__name__} is {ctypes.sizeof(st)} B in Python, {got} B in C")
        _LIB = handle
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().vs_last_error().decode() if rc == -1 else f"HIP error {rc}"
        raise VsError(f"{what}: {msg}")


def stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return VS_F32
    if dt == torch.bfloat16:
        return VS_BF16
    raise VsError(f"unsupported dtype {dt} (float32 / bfloat16 only)")


def require_device(*tensors) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise VsError("vspike ops run on the GPU only (tensor on %s); there is no CPU fallback" % t.device)


class BwdChain:
    """Owner of one vs_bwd_chain (side stream + deferred-join state of one backward sequence).
    Created on the current device; destroyed with the object."""

    def __init__(self):
        h = c_p()
        check(lib().vs_bwd_chain_create(ctypes.byref(h)), "vs_bwd_chain_create")
        self.handle = h.value

    def close(self):
        if getattr(self, "handle", None):
            lib().vs_bwd_chain_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def build_id() -> str:
    """vs_build_id() of the loaded library: the source hash it was compiled from (vspike.build.source_hash)."""
    return lib().vs_build_id().decode()


def dispatch_counts() -> dict:
    """Launches per kernel path since the last dispatch_reset() (vspike.h VS_PATH_*)."""
    buf = (c_i64 * PATH_COUNT)()
    lib().vs_dispatch_counts(buf, PATH_COUNT)
    return {name: int(buf[i]) for i, name in enumerate(PATH_NAMES)}


def dispatch_reset() -> None:
    lib().vs_dispatch_reset()


def attn_redo_count(reset: bool = False) -> int:
    """Workgroups of the bf16 attention forward that re-ran under the safe softmax (vs_attn_redo_count)."""
    v = c_i64()
    check(lib().vs_attn_redo_count(ctypes.byref(v), int(reset)), "vs_attn_redo_count")
    return int(v.value)


def knob_get(name: str) -> int:
    return int(lib().vs_knob_get(KNOB_NAMES.index(name)))


def knob_set(name: str, value: int) -> int:
    """Override an A/B knob (vspike.h VS_KNOB_*); returns the previous value."""
    return int(lib().vs_knob_set(KNOB_NAMES.index(name), int(value)))


def knobs_nondefault() -> dict:
    """Every knob whose current value differs from its built-in default (environment or
    vs_knob_set), plus "debug_knobs": 1 when the loaded library was built with VS_DEBUG_KNOBS
    (diagnostic variant whose timing knobs give wrong results).  Recorded by bench.py and smoke()."""
    h = lib()
    out = {name: int(h.vs_knob_get(i)) for i, name in enumerate(KNOB_NAMES)
           if int(h.vs_knob_get(i)) != int(h.vs_knob_default(i))}
    if int(h.vs_debug_knobs()):
        out["debug_knobs"] = 1
    return out


class knob:
    """Context manager: `with knob("no_wres", 1): ...` selects a kernel path for the block."""

    def __init__(self, name: str, value: int):
        self.name, self.value, self.prev = name, int(value), None

    def __enter__(self):
        self.prev = knob_set(self.name, self.value)
        return self

    def __exit__(self, *exc):
        knob_set(self.name, self.prev)
        return False
