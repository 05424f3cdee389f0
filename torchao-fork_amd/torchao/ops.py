"""``torch.ops.torchao`` operators of the MI355X weight-only quantized linear path.

Follows the reference's registration pattern (torchao/ops.py:12-21 ``Library("torchao",
"FRAGMENT")`` + ``lib.define`` schemas, :73-77 ``register_fake`` meta impls using
``torch._check``). The device impls are registered for the ``CUDA`` dispatch key (which is HIP
on ROCm, as in tensor_core_tiled_layout.cu:370-374) and call the gfx950 C-ABI library
(``include/torchao_mi355x.h``) on the current stream: no allocation besides the output (caching
allocator), no host synchronisation, so every op is hipGraph-capturable.

Operators:
  * ``unpack_tensor_core_tiled_layout`` / ``dequantize_tensor_core_tiled_layout`` — the
    reference schemas (ops.py:16-21) on the reference tile format, with an optional
    ``tile_format``: the CUDA nibble map of the reference's .cu kernels, or the one PyTorch-ROCm's
    ``aten._convert_weight_to_int4pack`` writes (the default on ROCm builds).
  * ``pack_tensor_core_tiled_layout`` — inverse of the unpack (bit-identical to
    ``aten._convert_weight_to_int4pack`` in the ROCm map), for checkpoint interchange.
  * ``int4_pack`` / ``int4_unpack`` / ``int4_dequantize`` / ``int4_weight_only_linear`` — the
    gfx950 row-stream int4 layout; ``int4_weight_only_linear`` replaces
    ``aten._weight_int4pack_mm`` (tensor_core_tiled_layout.py:104).
  * ``int8_weight_only_linear`` — replaces mm + scale (plain_layout.py:256-266).
  * ``int8_quantize_per_token`` / ``int8_scaled_mm`` — replace the activation quant
    (quant_api.py:1258-1273) and ``int_scaled_matmul`` + weight scale (plain_layout.py:294-315).
  * ``int8_dyn_linear`` — one token through both in one launch (decode), bit-identical.
  * ``int4_quantize_pack`` / ``int8_quantize_rows`` — the weight quantizers of
    ``from_hp_to_intx`` in one pass each (tinygemm qparams + quantize + row-stream pack;
    symmetric per-row int8), bit-exact to the bf16 torch-op formulation.
"""

import ctypes
import os
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchao import _lib

lib = torch.library.Library("torchao", "FRAGMENT")
# The reference schemas (ops.py:16-21) plus an optional trailing tile_format (-1 = this
# platform's aten format, see default_tile_format), so the reference's positional calls bind.
lib.define(
    "unpack_tensor_core_tiled_layout(Tensor packed_w, int inner_k_tiles, int tile_format=-1) "
    "-> Tensor"
)
lib.define(
    "dequantize_tensor_core_tiled_layout(Tensor packed_w, Tensor scales_and_zeros, "
    "int group_size, int inner_k_tiles, int tile_format=-1) -> Tensor"
)
lib.define(
    "pack_tensor_core_tiled_layout(Tensor int_data, int inner_k_tiles, int tile_format=-1) "
    "-> Tensor"
)
lib.define("int4_pack(Tensor int_data) -> Tensor")
lib.define("int4_pack_u8(Tensor int_data_u8) -> Tensor")
lib.define("int4_unpack(Tensor packed_w) -> Tensor")
lib.define(
    "int4_dequantize(Tensor packed_w, Tensor scales_and_zeros, int group_size, int mode=0) "
    "-> Tensor"
)
lib.define(
    "int4_weight_only_linear(Tensor x, Tensor packed_w, Tensor scales_and_zeros, "
    "int group_size, Tensor? bias=None) -> Tensor"
)
lib.define(
    "int8_weight_only_linear(Tensor x, Tensor w_int8, Tensor scale, Tensor? bias=None) -> Tensor"
)
lib.define("int8_quantize_per_token(Tensor x) -> (Tensor, Tensor)")
lib.define("int4_quantize_pack(Tensor w, int group_size, float eps) -> (Tensor, Tensor)")
lib.define("int8_quantize_rows(Tensor w, float eps) -> (Tensor, Tensor)")
lib.define(
    "int8_scaled_mm(Tensor x_int8, Tensor x_scale, Tensor w_int8, Tensor w_scale, "
    "Tensor? bias=None) -> Tensor"
)
lib.define(
    "int8_dyn_linear(Tensor x, Tensor w_int8, Tensor w_scale, Tensor? bias=None) -> Tensor"
)

_GROUP_SIZES = (32, 64, 128, 256)


def _ptr(t: Optional[Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(t: Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _require_contig(t: Tensor, name: str):
    torch._check(t.is_contiguous(), lambda: f"{name} must be contiguous")


def _same_device(x: Tensor, **operands):
    """Every operand on x's device (the kernels take raw device pointers; a tensor on another
    GPU or the host would reach the launch as a foreign pointer). RuntimeError otherwise, like
    the C++ op kernels (csrc/torch_ops.cpp check_device)."""
    for name, t in operands.items():
        if t is not None and t.device != x.device:
            raise RuntimeError(f"{name} is on {t.device} but x is on {x.device}: all operands "
                               "must be on the same device")


# ---------------------------------------------------------------------------------------------
# reference tile format (torchao/ops.py:255-377)
# ---------------------------------------------------------------------------------------------
TILE_FORMAT_CUDA = 0  # tensor_core_tiled_layout.cu:131-215 (aten on CUDA builds)
TILE_FORMAT_ROCM = 1  # aten._convert_weight_to_int4pack on PyTorch-ROCm (wave64 lanes)
_default_tile_format = TILE_FORMAT_ROCM if torch.version.hip else TILE_FORMAT_CUDA


def default_tile_format() -> int:
    """The nibble map ``aten._convert_weight_to_int4pack`` writes on this PyTorch build (both
    share the tile tensor's shape; include/torchao_mi355x.h documents the two maps)."""
    return _default_tile_format


def set_default_tile_format(fmt) -> None:
    """Select the map that tile_format=-1 means: "cuda" / 0 to read a TensorCoreTiledLayout
    checkpoint written by a CUDA build of torchao, "rocm" / 1 for one written on ROCm. This is
    also the explicit choice that lets reference checkpoints load (``checkpoint_tile_format``)."""
    global _default_tile_format, _chosen_tile_format
    _default_tile_format = _tile_format(fmt)
    _chosen_tile_format = _default_tile_format


# The map a reference checkpoint's tile storage is read with. The two maps share the tile
# tensor's shape and cannot be told apart from the bytes, and CUDA builds write most
# checkpoints, so loading never guesses: None until set_default_tile_format() or the
# checkpoint_tile_format() context chooses one.
_chosen_tile_format = None


class checkpoint_tile_format:
    """``with torchao.ops.checkpoint_tile_format("cuda"): torch.load(...)`` — the nibble map of
    the reference TensorCoreTiledLayout storage being loaded, for the duration of the block."""

    def __init__(self, fmt):
        self.fmt = _tile_format(fmt) if fmt != -1 else -1
        torch._check(self.fmt != -1, lambda: "checkpoint_tile_format needs 'cuda' or 'rocm'")

    def __enter__(self):
        global _chosen_tile_format
        self._prev = _chosen_tile_format
        _chosen_tile_format = self.fmt
        return self

    def __exit__(self, *exc):
        global _chosen_tile_format
        _chosen_tile_format = self._prev
        return False


def chosen_checkpoint_tile_format() -> int:
    """The explicitly chosen map for reference tile storage; raises if none was chosen."""
    if _chosen_tile_format is None:
        raise RuntimeError(
            "this checkpoint holds int4 weights in the reference's TensorCoreTiledLayout tile "
            "format, whose nibble map depends on the PyTorch build that wrote it (CUDA or ROCm) "
            "and cannot be detected from the bytes. Choose it before loading: "
            "torchao.ops.set_default_tile_format('cuda' | 'rocm'), or "
            "`with torchao.ops.checkpoint_tile_format('cuda' | 'rocm'): torch.load(...)`")
    return _chosen_tile_format


def _tile_format(fmt) -> int:
    if isinstance(fmt, str):
        fmt = {"cuda": TILE_FORMAT_CUDA, "rocm": TILE_FORMAT_ROCM}.get(fmt.lower(), -2)
    if fmt == -1:
        return _default_tile_format
    torch._check(fmt in (TILE_FORMAT_CUDA, TILE_FORMAT_ROCM),
                 lambda: f"tile_format must be 'cuda' (0), 'rocm' (1) or -1, got {fmt}")
    return int(fmt)


def _check_tile_n(N: int, fmt: int):
    if fmt == TILE_FORMAT_ROCM:
        torch._check(N % 16 == 0, lambda: f"ROCm tile format needs N % 16 == 0, got N={N}")


def _check_tile(packed_w: Tensor, inner_k_tiles: int):
    torch._check(
        packed_w.dim() == 4, lambda: f"packed weight should be a 4d tensor, got {packed_w.dim()}D"
    )
    torch._check(
        packed_w.dtype is torch.int32, lambda: f"weight must be INT32, got {packed_w.dtype}"
    )
    torch._check(inner_k_tiles in (2, 4, 8), lambda: "inner_k_tiles must be 2, 4, or 8")
    torch._check(packed_w.size(2) == 32, lambda: "packed weight must have 32 at dim 2")
    torch._check(
        packed_w.size(3) == inner_k_tiles // 2,
        lambda: "packed weight must have inner_k_tiles/2 at dim 3",
    )
    return packed_w.size(0) * 8, packed_w.size(1) * inner_k_tiles * 16


def _check_tile_sz(sz: Tensor, group_size: int, N: int, K: int):
    torch._check(sz.dtype is torch.bfloat16, lambda: "scales_and_zeros must be bfloat16")
    torch._check(sz.dim() == 3, lambda: f"scales_and_zeros must be 3D, got {sz.dim()}")
    torch._check(group_size in _GROUP_SIZES, lambda: "qGroupSize must be 32, 64, 128, or 256")
    torch._check(
        sz.size(0) == K // group_size, lambda: "scales_and_zeros must have K // qGroupSize at dim 0"
    )
    torch._check(sz.size(1) == N, lambda: "scales_and_zeros must have N at dim 1")
    torch._check(sz.size(2) == 2, lambda: "scales_and_zeros must have 2 at dim 2")


@torch.library.register_fake("torchao::unpack_tensor_core_tiled_layout")
def _(packed_w: Tensor, inner_k_tiles: int, tile_format: int = -1) -> Tensor:
    N, K = _check_tile(packed_w, inner_k_tiles)
    _check_tile_n(N, _tile_format(tile_format))
    return packed_w.new_empty((N, K), dtype=torch.int32)


def _unpack_tile_cuda(packed_w: Tensor, inner_k_tiles: int, tile_format: int = -1) -> Tensor:
    N, K = _check_tile(packed_w, inner_k_tiles)
    fmt = _tile_format(tile_format)
    _check_tile_n(N, fmt)
    _require_contig(packed_w, "packed_w")
    out = torch.empty((N, K), dtype=torch.int32, device=packed_w.device)
    with torch.cuda.device(packed_w.device):
        _lib.call("tao_unpack_tensor_core_tiled_layout", _ptr(packed_w), _ptr(out), N, K,
                  inner_k_tiles, fmt, _stream(packed_w))
    return out


def _unpack_tile_cpu(packed_w: Tensor, inner_k_tiles: int, tile_format: int = -1) -> Tensor:
    """Host C++ unpack (tao_unpack_tensor_core_tiled_layout_host) for CPU-resident checkpoints."""
    N, K = _check_tile(packed_w, inner_k_tiles)
    fmt = _tile_format(tile_format)
    _check_tile_n(N, fmt)
    packed_w = packed_w.contiguous()
    out = torch.empty((N, K), dtype=torch.int32)
    _lib.call("tao_unpack_tensor_core_tiled_layout_host", _ptr(packed_w), _ptr(out), N, K,
              inner_k_tiles, fmt)
    return out


@torch.library.register_fake("torchao::dequantize_tensor_core_tiled_layout")
def _(packed_w: Tensor, scales_and_zeros: Tensor, group_size: int, inner_k_tiles: int,
      tile_format: int = -1) -> Tensor:
    N, K = _check_tile(packed_w, inner_k_tiles)
    _check_tile_n(N, _tile_format(tile_format))
    _check_tile_sz(scales_and_zeros, group_size, N, K)
    return packed_w.new_empty((N, K), dtype=torch.bfloat16)


def _dequant_tile_cuda(packed_w, scales_and_zeros, group_size, inner_k_tiles, tile_format=-1):
    N, K = _check_tile(packed_w, inner_k_tiles)
    fmt = _tile_format(tile_format)
    _check_tile_n(N, fmt)
    _check_tile_sz(scales_and_zeros, group_size, N, K)
    _same_device(packed_w, scales_and_zeros=scales_and_zeros)
    _require_contig(packed_w, "packed_w")
    _require_contig(scales_and_zeros, "scales_and_zeros")
    out = torch.empty((N, K), dtype=torch.bfloat16, device=packed_w.device)
    with torch.cuda.device(packed_w.device):
        _lib.call("tao_dequantize_tensor_core_tiled_layout", _ptr(packed_w),
                  _ptr(scales_and_zeros), _ptr(out), N, K, group_size, inner_k_tiles, fmt,
                  _stream(packed_w))
    return out


def _check_pack_tile(int_data: Tensor, inner_k_tiles: int):
    torch._check(int_data.dim() == 2 and int_data.dtype is torch.int32,
                 lambda: "int_data must be a 2D int32 tensor")
    torch._check(inner_k_tiles in (2, 4, 8), lambda: "inner_k_tiles must be 2, 4, or 8")
    N, K = int_data.shape
    torch._check(N % 8 == 0, lambda: f"N ({N}) must be a multiple of 8")
    torch._check(K % (inner_k_tiles * 16) == 0,
                 lambda: f"K ({K}) must be a multiple of {inner_k_tiles * 16}")
    return N, K


@torch.library.register_fake("torchao::pack_tensor_core_tiled_layout")
def _(int_data: Tensor, inner_k_tiles: int, tile_format: int = -1) -> Tensor:
    N, K = _check_pack_tile(int_data, inner_k_tiles)
    _check_tile_n(N, _tile_format(tile_format))
    return int_data.new_empty(
        (N // 8, K // (inner_k_tiles * 16), 32, inner_k_tiles // 2), dtype=torch.int32
    )


def _pack_tile_cuda(int_data: Tensor, inner_k_tiles: int, tile_format: int = -1) -> Tensor:
    N, K = _check_pack_tile(int_data, inner_k_tiles)
    fmt = _tile_format(tile_format)
    _check_tile_n(N, fmt)
    _require_contig(int_data, "int_data")
    out = torch.empty((N // 8, K // (inner_k_tiles * 16), 32, inner_k_tiles // 2),
                      dtype=torch.int32, device=int_data.device)
    with torch.cuda.device(int_data.device):
        _lib.call("tao_pack_tensor_core_tiled_layout", _ptr(int_data), _ptr(out), N, K,
                  inner_k_tiles, fmt, _stream(int_data))
    return out


# ---------------------------------------------------------------------------------------------
# gfx950 row-stream int4 layout
# ---------------------------------------------------------------------------------------------
def _check_int4_plain(int_data: Tensor):
    torch._check(int_data.dim() == 2, lambda: "int4_pack expects a 2D [N, K] tensor")
    torch._check(int_data.dtype is torch.int32, lambda: "int4_pack expects int32 values 0..15")
    torch._check(int_data.size(1) % 8 == 0, lambda: "int4_pack: K must be a multiple of 8")


@torch.library.register_fake("torchao::int4_pack")
def _(int_data: Tensor) -> Tensor:
    _check_int4_plain(int_data)
    return int_data.new_empty((int_data.size(0), int_data.size(1) // 8), dtype=torch.int32)


def _int4_pack_cuda(int_data: Tensor) -> Tensor:
    _check_int4_plain(int_data)
    int_data = int_data.contiguous()
    N, K = int_data.shape
    out = torch.empty((N, K // 8), dtype=torch.int32, device=int_data.device)
    with torch.cuda.device(int_data.device):
        _lib.call("tao_int4_pack", _ptr(int_data), _ptr(out), N, K, _stream(int_data))
    return out


def _int4_pack_cpu(int_data: Tensor) -> Tensor:
    _check_int4_plain(int_data)
    int_data = int_data.contiguous()
    N, K = int_data.shape
    out = torch.empty((N, K // 8), dtype=torch.int32)
    _lib.call("tao_int4_pack_host", _ptr(int_data), _ptr(out), N, K)
    return out


@torch.library.register_fake("torchao::int4_pack_u8")
def _(int_data_u8: Tensor) -> Tensor:
    torch._check(int_data_u8.dim() == 2 and int_data_u8.dtype is torch.uint8,
                 lambda: "int4_pack_u8 expects a 2D uint8 [N, K/2] tensor")
    return int_data_u8.new_empty((int_data_u8.size(0), int_data_u8.size(1) // 4), dtype=torch.int32)


def _int4_pack_u8_cuda(int_data_u8: Tensor) -> Tensor:
    torch._check(int_data_u8.dim() == 2 and int_data_u8.dtype is torch.uint8,
                 lambda: "int4_pack_u8 expects a 2D uint8 [N, K/2] tensor")
    int_data_u8 = int_data_u8.contiguous()
    N, K = int_data_u8.size(0), int_data_u8.size(1) * 2
    out = torch.empty((N, K // 8), dtype=torch.int32, device=int_data_u8.device)
    with torch.cuda.device(int_data_u8.device):
        _lib.call("tao_int4_pack_u8", _ptr(int_data_u8), _ptr(out), N, K, _stream(int_data_u8))
    return out


@torch.library.register_fake("torchao::int4_unpack")
def _(packed_w: Tensor) -> Tensor:
    torch._check(packed_w.dim() == 2 and packed_w.dtype is torch.int32,
                 lambda: "int4_unpack expects a 2D int32 [N, K/8] tensor")
    return packed_w.new_empty((packed_w.size(0), packed_w.size(1) * 8), dtype=torch.int32)


def _int4_unpack_cuda(packed_w: Tensor) -> Tensor:
    _require_contig(packed_w, "packed_w")
    N, K = packed_w.size(0), packed_w.size(1) * 8
    out = torch.empty((N, K), dtype=torch.int32, device=packed_w.device)
    with torch.cuda.device(packed_w.device):
        _lib.call("tao_int4_unpack", _ptr(packed_w), _ptr(out), N, K, _stream(packed_w))
    return out


def _int4_unpack_cpu(packed_w: Tensor) -> Tensor:
    packed_w = packed_w.contiguous()
    N, K = packed_w.size(0), packed_w.size(1) * 8
    out = torch.empty((N, K), dtype=torch.int32)
    _lib.call("tao_int4_unpack_host", _ptr(packed_w), _ptr(out), N, K)
    return out


def _check_int4_weight(packed_w: Tensor, sz: Tensor, group_size: int):
    torch._check(packed_w.dim() == 2 and packed_w.dtype is torch.int32,
                 lambda: "packed weight must be a 2D int32 [N, K/8] tensor")
    N, K = packed_w.size(0), packed_w.size(1) * 8
    torch._check(group_size in _GROUP_SIZES, lambda: "qGroupSize must be 32, 64, 128, or 256")
    torch._check(K % group_size == 0, lambda: f"K ({K}) must be divisible by qGroupSize")
    torch._check(sz.dtype is torch.bfloat16, lambda: "scales_and_zeros must be bfloat16")
    torch._check(
        tuple(sz.shape) == (N, K // group_size, 2),
        lambda: f"scales_and_zeros must be [N, K/g, 2] = {(N, K // group_size, 2)}, got {tuple(sz.shape)}",
    )
    return N, K


@torch.library.register_fake("torchao::int4_dequantize")
def _(packed_w: Tensor, scales_and_zeros: Tensor, group_size: int, mode: int = 0) -> Tensor:
    N, K = _check_int4_weight(packed_w, scales_and_zeros, group_size)
    return packed_w.new_empty((N, K), dtype=torch.bfloat16)


def _int4_dequant_cuda(packed_w, scales_and_zeros, group_size, mode=0):
    N, K = _check_int4_weight(packed_w, scales_and_zeros, group_size)
    _same_device(packed_w, scales_and_zeros=scales_and_zeros)
    _require_contig(packed_w, "packed_w")
    _require_contig(scales_and_zeros, "scales_and_zeros")
    out = torch.empty((N, K), dtype=torch.bfloat16, device=packed_w.device)
    with torch.cuda.device(packed_w.device):
        _lib.call("tao_int4_dequant", _ptr(packed_w), _ptr(scales_and_zeros), _ptr(out), N, K,
                  group_size, int(mode), _stream(packed_w))
    return out


def _linear_out_shape(x: Tensor, N: int):
    return (*x.shape[:-1], N)


@torch.library.register_fake("torchao::int4_weight_only_linear")
def _(x, packed_w, scales_and_zeros, group_size, bias=None):
    N, K = _check_int4_weight(packed_w, scales_and_zeros, group_size)
    torch._check(x.dtype is torch.bfloat16, lambda: "int4 weight-only linear needs bf16 input")
    torch._check(x.size(-1) == K, lambda: f"x last dim {x.size(-1)} != K {K}")
    return x.new_empty(_linear_out_shape(x, N))


def _int4_linear_cuda(x, packed_w, scales_and_zeros, group_size, bias=None):
    N, K = _check_int4_weight(packed_w, scales_and_zeros, group_size)
    torch._check(x.dtype is torch.bfloat16, lambda: "int4 weight-only linear needs bf16 input")
    torch._check(x.size(-1) == K, lambda: f"x last dim {x.size(-1)} != K {K}")
    _same_device(x, packed_w=packed_w, scales_and_zeros=scales_and_zeros, bias=bias)
    x2 = x.reshape(-1, K)
    if not x2.is_contiguous() or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    M = x2.size(0)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
    _require_contig(packed_w, "packed_w")
    _require_contig(scales_and_zeros, "scales_and_zeros")
    with torch.cuda.device(x.device):
        _lib.call("tao_int4wo_linear_bf16", _ptr(x2), _ptr(packed_w), _ptr(scales_and_zeros),
                  _ptr(bias), _ptr(y), M, N, K, group_size, _stream(x))
    return y.reshape(_linear_out_shape(x, N))


# ---------------------------------------------------------------------------------------------
# int8 weight-only and dynamic activation
# ---------------------------------------------------------------------------------------------
def _check_int8_weight(w: Tensor, scale: Tensor):
    torch._check(w.dim() == 2 and w.dtype is torch.int8, lambda: "w must be a 2D int8 tensor")
    torch._check(scale.numel() == w.size(0), lambda: "scale must have N elements")
    return w.shape


@torch.library.register_fake("torchao::int8_weight_only_linear")
def _(x, w_int8, scale, bias=None):
    N, K = _check_int8_weight(w_int8, scale)
    torch._check(x.size(-1) == K, lambda: f"x last dim {x.size(-1)} != K {K}")
    return x.new_empty(_linear_out_shape(x, N))


def _int8wo_linear_cuda(x, w_int8, scale, bias=None):
    N, K = _check_int8_weight(w_int8, scale)
    torch._check(x.dtype is torch.bfloat16, lambda: "int8 weight-only linear (HIP) needs bf16 x")
    torch._check(x.size(-1) == K, lambda: f"x last dim {x.size(-1)} != K {K}")
    _same_device(x, w_int8=w_int8, scale=scale, bias=bias)
    x2 = x.reshape(-1, K)
    if not x2.is_contiguous() or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    M = x2.size(0)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    w_int8 = w_int8.contiguous()
    scale = scale.reshape(-1).to(torch.bfloat16).contiguous()
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
    with torch.cuda.device(x.device):
        _lib.call("tao_int8wo_linear_bf16", _ptr(x2), _ptr(w_int8), _ptr(scale), _ptr(bias),
                  _ptr(y), M, N, K, _stream(x))
    return y.reshape(_linear_out_shape(x, N))


@torch.library.register_fake("torchao::int8_quantize_per_token")
def _(x):
    return (
        x.new_empty(x.shape, dtype=torch.int8),
        x.new_empty((*x.shape[:-1], 1), dtype=torch.bfloat16),
    )


def _int8_quant_cuda(x: Tensor) -> Tuple[Tensor, Tensor]:
    torch._check(x.dtype is torch.bfloat16, lambda: "int8 per-token quant (HIP) needs bf16 x")
    K = x.size(-1)
    x2 = x.reshape(-1, K)
    if not x2.is_contiguous() or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    M = x2.size(0)
    q = torch.empty((M, K), dtype=torch.int8, device=x.device)
    s = torch.empty((M, 1), dtype=torch.bfloat16, device=x.device)
    with torch.cuda.device(x.device):
        _lib.call("tao_int8_quant_per_token", _ptr(x2), _ptr(q), _ptr(s), M, K, _stream(x))
    return q.reshape(x.shape), s.reshape(*x.shape[:-1], 1)


@torch.library.register_fake("torchao::int8_scaled_mm")
def _(x_int8, x_scale, w_int8, w_scale, bias=None):
    N, K = _check_int8_weight(w_int8, w_scale)
    return x_int8.new_empty(_linear_out_shape(x_int8, N), dtype=torch.bfloat16)


def _int8_scaled_mm_cuda(x_int8, x_scale, w_int8, w_scale, bias=None):
    N, K = _check_int8_weight(w_int8, w_scale)
    torch._check(x_int8.dtype is torch.int8, lambda: "x_int8 must be int8")
    torch._check(x_int8.size(-1) == K, lambda: f"x last dim {x_int8.size(-1)} != K {K}")
    _same_device(x_int8, x_scale=x_scale, w_int8=w_int8, w_scale=w_scale, bias=bias)
    x2 = x_int8.reshape(-1, K).contiguous()
    M = x2.size(0)
    xs = x_scale.reshape(-1).to(torch.bfloat16).contiguous()
    torch._check(xs.numel() == M, lambda: "x_scale must have one entry per row")
    ws = w_scale.reshape(-1).to(torch.bfloat16).contiguous()
    w_int8 = w_int8.contiguous()
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x_int8.device)
    with torch.cuda.device(x_int8.device):
        _lib.call("tao_int8_scaled_mm_bf16", _ptr(x2), _ptr(xs), _ptr(w_int8), _ptr(ws),
                  _ptr(bias), _ptr(y), M, N, K, _stream(x_int8))
    return y.reshape(_linear_out_shape(x_int8, N))


@torch.library.register_fake("torchao::int8_dyn_linear")
def _(x, w_int8, w_scale, bias=None):
    N, K = _check_int8_weight(w_int8, w_scale)
    torch._check(x.numel() == K, lambda: "int8_dyn_linear is one token (x.numel() == K)")
    return x.new_empty(_linear_out_shape(x, N), dtype=torch.bfloat16)


def _int8_dyn_linear_cuda(x, w_int8, w_scale, bias=None):
    """One token: per-token int8 quant + int8 x int8 GEMV in one launch, bit-identical to
    int8_quantize_per_token -> int8_scaled_mm."""
    N, K = _check_int8_weight(w_int8, w_scale)
    torch._check(x.dtype is torch.bfloat16, lambda: "int8_dyn_linear (HIP) needs bf16 x")
    torch._check(x.size(-1) == K, lambda: f"x last dim {x.size(-1)} != K {K}")
    torch._check(x.numel() == K, lambda: "int8_dyn_linear is one token (x.numel() == K)")
    _same_device(x, w_int8=w_int8, w_scale=w_scale, bias=bias)
    x2 = x.reshape(1, K)
    if not x2.is_contiguous() or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    ws = w_scale.reshape(-1).to(torch.bfloat16).contiguous()
    w_int8 = w_int8.contiguous()
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
    y = torch.empty((1, N), dtype=torch.bfloat16, device=x.device)
    with torch.cuda.device(x.device):
        _lib.call("tao_int8_dyn_linear_bf16", _ptr(x2), _ptr(w_int8), _ptr(ws), _ptr(bias),
                  _ptr(y), 1, N, K, _stream(x))
    return y.reshape(_linear_out_shape(x, N))


@torch.library.register_fake("torchao::int4_quantize_pack")
def _(w, group_size, eps):
    torch._check(group_size in _GROUP_SIZES, lambda: "group_size must be 32, 64, 128, or 256")
    K = w.size(-1)
    torch._check(K % group_size == 0, lambda: f"K ({K}) must be divisible by group_size")
    lead = w.shape[:-1]
    return (w.new_empty((*lead, K // 8), dtype=torch.int32),
            w.new_empty((*lead, K // group_size, 2), dtype=torch.bfloat16))


def _int4_quantize_pack_cuda(w: Tensor, group_size: int, eps: float):
    """bf16 W [..., K] -> (packed int32 [..., K/8], scales_and_zeros bf16 [..., K/g, 2])."""
    torch._check(w.dtype is torch.bfloat16, lambda: "int4 quantize (HIP) needs a bf16 weight")
    torch._check(group_size in _GROUP_SIZES, lambda: "group_size must be 32, 64, 128, or 256")
    K = w.size(-1)
    torch._check(K % group_size == 0, lambda: f"K ({K}) must be divisible by group_size")
    w2 = w.reshape(-1, K)
    if not w2.is_contiguous() or w2.data_ptr() % 16:
        w2 = w2.contiguous()
    R = w2.size(0)
    packed = torch.empty((R, K // 8), dtype=torch.int32, device=w.device)
    sz = torch.empty((R, K // group_size, 2), dtype=torch.bfloat16, device=w.device)
    with torch.cuda.device(w.device):
        _lib.call("tao_int4_quantize_bf16", _ptr(w2), _ptr(packed), _ptr(sz), R, K, group_size,
                  ctypes.c_float(eps), _stream(w))
    lead = w.shape[:-1]
    return packed.reshape(*lead, K // 8), sz.reshape(*lead, K // group_size, 2)


@torch.library.register_fake("torchao::int8_quantize_rows")
def _(w, eps):
    return (w.new_empty(w.shape, dtype=torch.int8),
            w.new_empty(w.shape[:-1], dtype=torch.bfloat16))


def _int8_quantize_rows_cuda(w: Tensor, eps: float):
    """bf16 W [..., K] -> (int8 [..., K], per-row scale bf16 [...]), symmetric [-128, 127]."""
    torch._check(w.dtype is torch.bfloat16, lambda: "int8 quantize (HIP) needs a bf16 weight")
    K = w.size(-1)
    torch._check(K % 8 == 0, lambda: f"K ({K}) must be a multiple of 8")
    w2 = w.reshape(-1, K)
    if not w2.is_contiguous() or w2.data_ptr() % 16:
        w2 = w2.contiguous()
    R = w2.size(0)
    q = torch.empty((R, K), dtype=torch.int8, device=w.device)
    s = torch.empty((R,), dtype=torch.bfloat16, device=w.device)
    with torch.cuda.device(w.device):
        _lib.call("tao_int8_quantize_rows_bf16", _ptr(w2), _ptr(q), _ptr(s), R, K,
                  ctypes.c_float(eps), _stream(w))
    return q.reshape(w.shape), s.reshape(w.shape[:-1])


# ---- register device impls ------------------------------------------------------------------
# The per-linear ops take their CUDA kernels from libtorchao_ops.so (csrc/torch_ops.cpp: the
# same checks, then the C-ABI, with no Python frame: ~19 -> ~7 µs of host time per call at
# M = 1, profiles/r2_eager_overhead*.json). The Python impls below serve the rest, and these
# too when that library cannot load or an experiment points TORCHAO_MI355X_LIB at a variant
# build (the C++ kernels are linked to the in-tree library).
_OPS_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtorchao_ops.so")
_native_served: frozenset = frozenset()
_native_error: Optional[str] = None
if os.environ.get("TORCHAO_MI355X_LIB"):
    _native_error = "TORCHAO_MI355X_LIB is set (variant build): Python impls"
else:
    try:
        torch.ops.load_library(_OPS_LIB)
        _served = ctypes.CDLL(_OPS_LIB).tao_torch_ops_served
        _served.restype = ctypes.c_char_p
        _native_served = frozenset(_served().decode().split(","))
    except (OSError, RuntimeError, AttributeError) as e:
        _native_error = f"{type(e).__name__}: {e}"


def native_dispatch() -> frozenset:
    """The ``torch.ops.torchao`` ops whose CUDA kernel is C++ (libtorchao_ops.so)."""
    return _native_served


for _name, _fn in [
    ("unpack_tensor_core_tiled_layout", _unpack_tile_cuda),
    ("dequantize_tensor_core_tiled_layout", _dequant_tile_cuda),
    ("pack_tensor_core_tiled_layout", _pack_tile_cuda),
    ("int4_pack", _int4_pack_cuda),
    ("int4_pack_u8", _int4_pack_u8_cuda),
    ("int4_unpack", _int4_unpack_cuda),
    ("int4_dequantize", _int4_dequant_cuda),
    ("int4_weight_only_linear", _int4_linear_cuda),
    ("int8_weight_only_linear", _int8wo_linear_cuda),
    ("int8_quantize_per_token", _int8_quant_cuda),
    ("int4_quantize_pack", _int4_quantize_pack_cuda),
    ("int8_quantize_rows", _int8_quantize_rows_cuda),
    ("int8_scaled_mm", _int8_scaled_mm_cuda),
    ("int8_dyn_linear", _int8_dyn_linear_cuda),
]:
    if _name not in _native_served:
        lib.impl(_name, _fn, "CUDA")
# Host packers (C++ in the same library) so quantize_ works on CPU-resident models.
lib.impl("int4_pack", _int4_pack_cpu, "CPU")
lib.impl("int4_unpack", _int4_unpack_cpu, "CPU")
lib.impl("unpack_tensor_core_tiled_layout", _unpack_tile_cpu, "CPU")


# ---- Python-level wrappers with the reference names (ops.py:255-377) ------------------------
def unpack_tensor_core_tiled_layout(packed_w: Tensor, inner_k_tiles: int,
                                    tile_format=-1) -> Tensor:
    """Tile-format int4 weight [N/8][K/(ikt*16)][32][ikt/2] -> int32 [N, K]."""
    return torch.ops.torchao.unpack_tensor_core_tiled_layout.default(
        packed_w, inner_k_tiles, _tile_format(tile_format))


def dequantize_tensor_core_tiled_layout(
    packed_w: Tensor, scales_and_zeros: Tensor, group_size: int, inner_k_tiles: int,
    tile_format=-1,
) -> Tensor:
    """Tile-format int4 weight + [K/g, N, 2] scales/zeros -> bf16 [N, K]."""
    return torch.ops.torchao.dequantize_tensor_core_tiled_layout.default(
        packed_w, scales_and_zeros, group_size, inner_k_tiles, _tile_format(tile_format)
    )


def pack_tensor_core_tiled_layout(int_data: Tensor, inner_k_tiles: int,
                                  tile_format=-1) -> Tensor:
    """int32 [N, K] -> the tile format (tile_format 1 == PyTorch-ROCm's
    aten._convert_weight_to_int4pack of the same nibbles, bit for bit)."""
    return torch.ops.torchao.pack_tensor_core_tiled_layout.default(
        int_data, inner_k_tiles, _tile_format(tile_format))


def int4_weight_only_linear(x, packed_w, scales_and_zeros, group_size, bias=None):
    return torch.ops.torchao.int4_weight_only_linear.default(
        x, packed_w, scales_and_zeros, group_size, bias
    )
