"""ctypes binding of libspotter_hip.so (include/spotter_hip.h).

The product path has no fallback: if the library is missing or the device is
not gfx950, `lib()` raises. Every wrapper raises RuntimeError with
sp_last_error() on a non-zero status, so the unchanged AmenitiesDetector turns a
kernel failure into its per-image "Processing Error" (serve.py:152-157).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPOTTER_HIP_LIB", os.path.join(HERE, "libspotter_hip.so"))
ABI_VERSION = 15

vp = C.c_void_p
i32 = C.c_int32
i64 = C.c_int64
f32 = C.c_float


class SpImageU8(C.Structure):
    _fields_ = [("data", vp), ("height", i32), ("width", i32), ("row_stride", i32)]


class SpConvDesc(C.Structure):
    _fields_ = [
        ("A", vp), ("lda", i64), ("A2", vp), ("lda2", i64),
        ("N", i32), ("H", i32), ("W", i32), ("Cin", i32),
        ("KH", i32), ("KW", i32), ("stride", i32), ("pad", i32),
        ("Ho", i32), ("Wo", i32),
        ("Wt", vp), ("Cout", i32),
        ("scale", vp), ("shift", vp),
        ("row_scale", vp), ("row_period", i32),
        ("res1", vp), ("ldr1", i64),
        ("act", i32),
        ("res2", vp), ("ldr2", i64),
        ("C", vp), ("ldc", i64),
        ("out_rows_per_group", i32), ("out_group_stride", i64),
        ("workspace", vp), ("workspace_elems", i64),
        ("precision", i32), ("Wt_bf16", vp), ("wt_plane_stride", i64),
        ("ln_gamma", vp), ("ln_beta", vp), ("ln_eps", f32),
        ("A_bf16", vp),
        ("C_bf16", vp), ("res1_bf16", vp), ("res2_bf16", vp),
        ("splitk_counters", vp), ("splitk_counters_len", i64),
    ]


class SpMsdaDesc(C.Structure):
    _fields_ = [
        ("value", vp), ("ld_value", i64), ("value_col", i32),
        ("off_aw", vp), ("ld_off_aw", i64),
        ("ref", vp),
        ("out", vp), ("ld_out", i64),
        ("B", i32), ("S", i32), ("Q", i32), ("heads", i32), ("head_dim", i32),
        ("levels", i32), ("points", i32),
        ("level_h", i32 * 4), ("level_w", i32 * 4), ("level_start", i32 * 4),
        ("offset_scale", f32),
        ("value_bf16", vp),
    ]


class SpJpegLayout(C.Structure):
    _fields_ = [
        ("width", i32), ("height", i32), ("ncomp", i32), ("color", i32), ("progressive", i32),
        ("max_h", i32), ("max_v", i32), ("h", i32 * 3), ("v", i32 * 3), ("bw", i32 * 3), ("bh", i32 * 3),
        ("block_off", i64 * 3), ("total_blocks", i64), ("plane_off", i64 * 3), ("plane_bytes", i64),
        ("quant", (C.c_uint16 * 64) * 3),
    ]


class SpJpegEncLayout(C.Structure):
    _fields_ = [
        ("width", i32), ("height", i32), ("quality", i32), ("h0", i32), ("v0", i32),
        ("mcux", i32), ("mcuy", i32), ("bpm", i32), ("wb0", i32), ("hb0", i32),
        ("total_blocks", i64), ("work_bytes", i64), ("bits_cap", i64),
        ("quant", (C.c_uint16 * 64) * 2), ("recip", (C.c_uint16 * 64) * 2), ("corr", (C.c_uint16 * 64) * 2),
        ("shift", (C.c_int16 * 64) * 2),
    ]


SP_JPEG_UNSUPPORTED = -10
SP_BUILD_FUSED_LN = 1  # sp_build_flags bits (include/spotter_hip.h)
SP_BUILD_BOUNDS = 2

_SIGS = {
    "sp_abi_version": (i32, []),
    "sp_build_flags": (i32, []),
    "sp_bounds_report": (i64, [C.c_char_p, i64]),
    "sp_last_error": (C.c_char_p, []),
    "sp_device_init": (i32, [i32]),
    "sp_shutdown": (i32, []),
    "sp_preprocess_u8": (i32, [C.POINTER(SpImageU8), i32, i32, i32, vp, vp]),
    "sp_conv2d": (i32, [C.POINTER(SpConvDesc), vp]),
    "sp_set_conv_config": (i32, [i32]),
    "sp_set_splitk_config": (i32, [i32, i32, i32]),
    "sp_set_tuning": (i32, [i32, i32]),
    "sp_conv3x3_winograd": (i32, [C.POINTER(SpConvDesc), vp, i64, vp, i64, vp]),
    "sp_winograd_f23_input": (i32, [C.POINTER(SpConvDesc), vp, i64, vp]),
    "sp_winograd_f23_gemm": (i32, [C.POINTER(SpConvDesc), vp, i64, vp, i64, vp]),
    "sp_winograd_f23_output": (i32, [C.POINTER(SpConvDesc), vp, i64, vp]),
    "sp_winograd_f43_input": (i32, [C.POINTER(SpConvDesc), vp, i64, vp]),
    "sp_winograd_f43_gemm": (i32, [C.POINTER(SpConvDesc), vp, i64, vp, i64, vp]),
    "sp_winograd_f43_output": (i32, [C.POINTER(SpConvDesc), vp, i64, vp]),
    "sp_nchw_to_nhwc": (i32, [vp, vp, i32, i32, i32, i32, vp]),
    "sp_stem_conv3x3s2_nchw": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "sp_maxpool3x3s2": (i32, [vp, vp, i64, i32, i32, i32, i32, vp]),
    "sp_avgpool2x2_ceil": (i32, [vp, vp, i64, i32, i32, i32, i32, vp]),
    "sp_maxpool3x3s2_bf16": (i32, [vp, vp, i64, i32, i32, i32, i32, vp]),
    "sp_avgpool2x2_ceil_bf16": (i32, [vp, vp, i64, i32, i32, i32, i32, vp]),
    "sp_stem_conv3x3s2_nchw_bf16": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "sp_conv3x3_c32_bf16": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "sp_conv3x3_c32": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "sp_conv3x3_c64_bf16": (i32, [vp, i64, vp, vp, vp, vp, i64, vp, i64, i32, i32, i32, i32, vp]),
    "sp_upsample2x_nearest": (i32, [vp, i64, vp, i64, i32, i32, i32, i32, vp]),
    "sp_layernorm": (i32, [vp, i64, vp, vp, vp, i64, i32, i32, f32, vp]),
    "sp_layernorm_bf16": (i32, [vp, i64, vp, vp, vp, i64, i32, i32, f32, vp]),
    "sp_attention": (i32, [vp, i64, vp, i64, vp, i64, vp, i64, i32, i32, i32, i32, f32, vp]),
    "sp_attention_bf16": (i32, [vp, i64, vp, i64, vp, i64, vp, i64, i32, i32, i32, i32, f32, vp]),
    "sp_msda": (i32, [C.POINTER(SpMsdaDesc), vp]),
    "sp_topk_rows": (i32, [vp, i64, i32, i32, i32, i32, i32, vp, vp, vp]),
    "sp_rowmax": (i32, [vp, i64, i64, i32, vp, vp]),
    "sp_gather_rows": (i32, [vp, i64, i32, vp, i32, i32, i32, vp, i64, vp]),
    "sp_ref_init": (i32, [vp, i64, vp, vp, i32, i32, vp, vp]),
    "sp_box_refine": (i32, [vp, i64, vp, i32, vp]),
    "sp_add_rows": (i32, [vp, i64, vp, i64, vp, vp, i64, i32, i32, vp]),
    "sp_linear_rowmax_bf16": (i32, [vp, i64, vp, vp, i32, i32, i32, vp, vp]),
    "sp_postprocess": (i32, [vp, vp, vp, i32, i32, i32, i32, f32, vp, vp, vp, vp, vp, vp]),
    "sp_jpeg_decode_coefs": (i32, [vp, i64, C.POINTER(SpJpegLayout), vp, i64]),
    "sp_jpeg_to_rgb": (i32, [vp, C.POINTER(SpJpegLayout), vp, i64, vp, i64, vp, vp]),
    "sp_jpeg_enc_plan": (i32, [i32, i32, i32, i32, C.POINTER(SpJpegEncLayout)]),
    "sp_jpeg_enc_rgb": (i32, [vp, i64, i32, C.POINTER(SpJpegEncLayout), vp, i64, vp, i64, vp, vp]),
    "sp_jpeg_enc_max_bytes": (i64, [C.POINTER(SpJpegEncLayout), i64, i64]),
    "sp_jpeg_enc_finish": (i32, [C.POINTER(SpJpegEncLayout), vp, i64, vp, i64, vp, i64, C.POINTER(i64)]),
}

EXPORTS = tuple(_SIGS)

_lock = threading.Lock()
_lib = None


def load(path: str = LIB_PATH):
    """dlopen the library and bind every export (no device calls)."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"libspotter_hip.so not found at {path}; build it with `python -m spotter_amd.build_ext` "
            "(there is no CPU fallback)")
    L = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.sp_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libspotter_hip ABI {L.sp_abi_version()} != {ABI_VERSION}")
    return L


def lib():
    global _lib
    with _lock:
        if _lib is None:
            _lib = load()
        return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().sp_last_error().decode(errors="replace")
        raise RuntimeError(f"spotter_hip {what} failed ({rc}): {msg}")


def call(name: str, *args):
    check(getattr(lib(), name)(*args), name)
