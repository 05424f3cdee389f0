"""ctypes binding of the gfx950 C-ABI library (``include/torchao_mi355x.h``).

The reference loads its native ops as ``torchao/_C*.so`` through ``torch.ops.load_library``
(torchao/__init__.py:26-32). Here the native code is a plain C-ABI shared library with no torch
types in its signatures; this module binds it with ctypes and ``torchao.ops`` registers the
``torch.ops.torchao.*`` operators on top of it.

The product path never falls back to anything else: if the library is missing or was built
without a GPU-usable runtime, every op that needs it raises ``RuntimeError``.
"""

import ctypes
import os
from typing import Optional

_LIB_NAME = "libtorchao_mi355x.so"
# TORCHAO_MI355X_LIB overrides the in-tree build (experiment variants)
_LIB_PATH = os.environ.get("TORCHAO_MI355X_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), _LIB_NAME
)

_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[str] = None

_i64 = ctypes.c_int64
_p = ctypes.c_void_p
_int = ctypes.c_int

# name -> argtypes (restype is c_int unless listed in _RESTYPES)
_SIGNATURES = {
    "tao_version": [],
    "tao_last_error": [],
    "tao_last_kernel": [],
    "tao_device_count": [],
    "tao_profile_begin": [_int],
    "tao_profile_end": [_p, _int, _p],
    "tao_int4wo_linear_bf16": [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p],
    "tao_int4wo_linear_swiglu_bf16": [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _p],
    "tao_int4wo_linear_rope_kv_bf16": [_p, _p, _p, _i64, _i64, _p, _p, _p, _p, _p, _i64, _i64,
                                       _i64, _i64, _i64, _i64, _p],
    "tao_tune_int4_gemv": [_int, _int, _int, _int],
    "tao_tune_int4_lds": [_int],
    "tao_tune_linear_crossover": [_int],
    "tao_tune_gemm": [_int, _int, _int],
    "tao_tune_gemm_algo": [_int],
    "tao_tune_gemm_depth": [_int],
    "tao_tune_gemm_bn": [_int],
    "tao_tune_gemm_order": [_int],
    "tao_tune_gemm_nw": [_int],
    "tao_tune_gemm_table": [_int],
    "tao_tune_int4_mfma32": [_int],
    "tao_tune_int4_xlds": [_int],
    "tao_tune_int4_norm": [_int],
    "tao_tune_reset": [],
    "tao_tune_splitk_fenced": [_int],
    "tao_query_splitk_fenced": [],
    "tao_tune_gemm_tile": [_int, _int],
    "tao_tune_gemm_sf": [_int, _int, _int, _int, _int, _int, _int],
    "tao_gemm_sf_status": [_p],
    "tao_tune_gemm_sf_seam": [_int],
    "tao_tune_gemm_sf_loaders": [_int],
    "tao_tune_gemm_sf_xmap": [_int],
    "tao_tune_attn_prefill_nw": [_int],
    "tao_debug_sf_late_publisher": [_int],
    "tao_tune_cnt_stride": [_int],
    "tao_hbm_read_probe": [_p, _i64, _p, _p],
    "tao_hbm_copy_probe": [_p, _p, _i64, _int, _int, _p],
    "tao_sf_intake_probe": [_int, _int, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _p, _p],
    "tao_graph_workspace_count": [],
    "tao_int4_pack": [_p, _p, _i64, _i64, _p],
    "tao_int4_pack_u8": [_p, _p, _i64, _i64, _p],
    "tao_int4_unpack": [_p, _p, _i64, _i64, _p],
    "tao_int4_dequant": [_p, _p, _p, _i64, _i64, _i64, _int, _p],
    "tao_int4_pack_host": [_p, _p, _i64, _i64],
    "tao_int4_unpack_host": [_p, _p, _i64, _i64],
    "tao_unpack_tensor_core_tiled_layout": [_p, _p, _i64, _i64, _i64, _int, _p],
    "tao_unpack_tensor_core_tiled_layout_host": [_p, _p, _i64, _i64, _i64, _int],
    "tao_dequantize_tensor_core_tiled_layout": [_p, _p, _p, _i64, _i64, _i64, _i64, _int, _p],
    "tao_pack_tensor_core_tiled_layout": [_p, _p, _i64, _i64, _i64, _int, _p],
    "tao_int8wo_linear_bf16": [_p, _p, _p, _p, _p, _i64, _i64, _i64, _p],
    "tao_int8_quant_per_token": [_p, _p, _p, _i64, _i64, _p],
    "tao_int8_scaled_mm_bf16": [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p],
    "tao_int8_dyn_linear_bf16": [_p, _p, _p, _p, _p, _i64, _i64, _i64, _p],
    "tao_tune_int8_gemv": [_int, _int, _int],
    "tao_tune_int8_quant": [_int],
    "tao_rmsnorm_bf16": [_p, _p, _p, _i64, _i64, ctypes.c_float, _p],
    "tao_add_rmsnorm_bf16": [_p, _p, _p, _p, _p, _i64, _i64, ctypes.c_float, _p],
    "tao_add_rmsnorm_partials_bf16": [_p, _p, _i64, _p, _p, _p, _i64, _i64, ctypes.c_float, _p],
    "tao_int4wo_linear_partial_slices": [_i64, _i64, _i64, _i64, _p],
    "tao_int4wo_linear_partials_f32": [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _p],
    "tao_rope_kv_bf16": [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64, _p],
    "tao_attn_decode_split_bf16": [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64,
                                   ctypes.c_float, _i64, _p],
    "tao_attn_merge_bf16": [_p, _p, _i64, _i64, _i64, _i64, _p],
    "tao_int4wo_attn_out_bf16": [_p, _i64, _i64, _p, _p, _i64, _i64, _i64, _p, _p, _p],
    "tao_attn_decode_bf16": [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64,
                             ctypes.c_float, _p],
    "tao_attn_prefill_bf16": [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i64,
                              ctypes.c_float, _p],
    "tao_tune_attn": [_int],
    "tao_decode_status": [_p],
    "tao_silu_mul_bf16": [_p, _p, _p, _i64, _p],
    "tao_argmax_bf16": [_p, _p, _i64, _i64, _p],
    "tao_argmax_advance_bf16": [_p, _i64, _p, _p, _p, _i64, _p],
    "tao_int4_quantize_bf16": [_p, _p, _p, _i64, _i64, _i64, ctypes.c_float, _p],
    "tao_int8_quantize_rows_bf16": [_p, _p, _p, _i64, _i64, ctypes.c_float, _p],
    "tao_int4wo_grouped_gemv_bf16": [_p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _p, _p],
    "tao_int4wo_qkv_attn_supported": [_i64, _i64, _i64, _i64, _i64],
    "tao_int4wo_qkv_attn_bf16": [_p, _p, _p, _i64, _i64, _i64, _p, ctypes.c_float, _p, _p, _p,
                                 _p, _p, _p, _i64, _i64, _i64, _i64, ctypes.c_float, _i64, _p],
    "tao_int4wo_ffn_engine_supported": [_i64, _i64, _i64],
    "tao_debug_ffn_engine_stamps": [_p],
    "tao_tune_ffn_engine": [_int, _int, _int, _int],
    "tao_int4wo_ffn_engine_workspace_bytes": [_i64],
    "tao_int4wo_ffn_engine_bf16": [_p, _p, ctypes.c_float, _p, _p, _p, _p, _p, _i64, _i64, _i64,
                                   _p, _p, _p],
    "tao_int4wo_decode_bf16": [_p, _p, _p, _i64, _i64, _i64, _p, ctypes.c_float, _int, _p, _p,
                               _p, _p, _p, _i64, _i64, _i64, _i64, _p],
    "tao_int8wo_decode_bf16": [_p, _p, _p, _i64, _i64, _p, ctypes.c_float, _int, _p, _p, _p, _p, _p,
                               _i64, _i64, _i64, _i64, _p],
    "tao_int8dq_decode_bf16": [_p, _p, _p, _i64, _i64, _p, ctypes.c_float, _int, _p, _p, _p, _p, _p,
                               _i64, _i64, _i64, _i64, _p],
}
_RESTYPES = {"tao_version": ctypes.c_char_p, "tao_last_error": ctypes.c_char_p,
             "tao_last_kernel": ctypes.c_char_p,
             "tao_int4wo_ffn_engine_workspace_bytes": ctypes.c_int64}


def library_path() -> str:
    return _LIB_PATH


def exported_symbols():
    """Names the header declares (the C-ABI contract checked by the CPU tests)."""
    return sorted(_SIGNATURES)


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _load_error
    if _lib is not None or _load_error is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        _load_error = (
            f"{_LIB_NAME} not found at {_LIB_PATH}; build it with "
            "`make -C torchao-fork_amd/csrc` (or __graft_entry__.build())"
        )
        return None
    try:
        # torch must be imported first so the HIP runtime it bundles (same soname,
        # libamdhip64.so.7) is the one this library binds to.
        import torch  # noqa: F401

        lib = ctypes.CDLL(_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - environment specific
        _load_error = f"failed to load {_LIB_PATH}: {e}"
        return None
    for name, argtypes in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    _lib = lib
    return _lib


def is_available() -> bool:
    return _load() is not None


def load_error() -> Optional[str]:
    _load()
    return _load_error


def lib() -> ctypes.CDLL:
    """The loaded library; raises RuntimeError (never falls back) when it is missing."""
    handle = _load()
    if handle is None:
        raise RuntimeError(f"torchao MI355X native library unavailable: {_load_error}")
    return handle


class KernelTimer:
    """``with KernelTimer(n) as t: <launch kernels>`` -> ``t.durations_ms`` (one per launch).

    Uses tao_profile_begin/end: HIP events written by each kernel's own dispatch packet, so the
    numbers are kernel execution times (what rocprofv3 reports), without launch gaps."""

    def __init__(self, capacity: int):
        self.capacity = capacity
        self.durations_ms = []

    def __enter__(self):
        call("tao_profile_begin", self.capacity)
        return self

    def __exit__(self, *exc):
        buf = (ctypes.c_float * self.capacity)()
        n = ctypes.c_int(0)
        call("tao_profile_end", ctypes.cast(buf, ctypes.c_void_p), self.capacity,
             ctypes.cast(ctypes.pointer(n), ctypes.c_void_p))
        self.durations_ms = [float(buf[i]) for i in range(n.value)]
        return False


def call(name: str, *args) -> None:
    """Invoke a C-ABI entry point and turn a non-zero status into RuntimeError."""
    handle = lib()
    rc = getattr(handle, name)(*args)
    if rc != 0:
        msg = handle.tao_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")
