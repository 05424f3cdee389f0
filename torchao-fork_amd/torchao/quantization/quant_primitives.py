"""Affine quantization primitives for the weight-only / dynamic int8 linear path.

Restates the subset of the reference ``torchao/quantization/quant_primitives.py`` the hot path
uses, with identical names, arguments and floating-point op order (results are pinned
bit-for-bit against fixtures generated from the reference, tests/golden/):

  * ``choose_qparams_affine``            (reference :1497-1577, SYMMETRIC / ASYMMETRIC)
  * ``_choose_qparams_affine_tinygemm``  (:1238-1307; scale/zero in the input dtype)
  * ``quantize_affine``                  (:398-459; ``clamp(round(x * (1/s)) + zp)``)
  * ``_quantize_affine_tinygemm``        (:461-573; ``clamp(round((x - (z - s*mid)) / s))``)
  * ``_quantize_affine_no_zero_point``   (:600-690)
  * ``dequantize_affine`` / ``_dequantize_affine_tinygemm`` / ``_dequantize_affine_no_zero_point``
    (:779-1031)

These run with torch ops on whatever device the weight lives on: they execute once at
quantization time, outside the per-token hot loop (which is the HIP kernels behind torchao.ops).
"""

from enum import Enum, auto
from typing import List, Optional, Tuple, Union

import torch

__all__ = [
    "MappingType",
    "ZeroPointDomain",
    "choose_qparams_affine",
    "quantize_affine",
    "dequantize_affine",
    "_choose_qparams_affine_tinygemm",
    "_choose_qparams_affine_dont_preserve_zero",
    "_quantize_affine_tinygemm",
    "_dequantize_affine_tinygemm",
    "_quantize_affine_no_zero_point",
    "_dequantize_affine_no_zero_point",
    "_get_reduction_params",
]


class MappingType(Enum):
    """How float values map onto the integer grid (reference quant_primitives.py:61-80)."""

    SYMMETRIC = auto()
    SYMMETRIC_NO_CLIPPING_ERR = auto()
    ASYMMETRIC = auto()


class ZeroPointDomain(Enum):
    """Where the zero point lives: integer grid, float domain (tinygemm), or absent."""

    INT = auto()
    FLOAT = auto()
    NONE = auto()


_DTYPE_TO_QVALUE_BOUNDS = {
    torch.uint8: (0, 255),
    torch.int8: (-128, 127),
    torch.int16: (-(2**15), 2**15 - 1),
    torch.int32: (-(2**31), 2**31 - 1),
}
for _bits in range(1, 8):
    _u = getattr(torch, f"uint{_bits}", None)
    _s = getattr(torch, f"int{_bits}", None)
    if _u is not None:
        _DTYPE_TO_QVALUE_BOUNDS[_u] = (0, 2**_bits - 1)
    if _s is not None:
        _DTYPE_TO_QVALUE_BOUNDS[_s] = (-(2 ** (_bits - 1)), 2 ** (_bits - 1) - 1)


def _get_and_check_qmin_qmax(dtype, quant_min, quant_max):
    if dtype not in _DTYPE_TO_QVALUE_BOUNDS:
        raise ValueError(f"Unsupported dtype: {dtype}")
    lo, hi = _DTYPE_TO_QVALUE_BOUNDS[dtype]
    quant_min = lo if quant_min is None else quant_min
    quant_max = hi if quant_max is None else quant_max
    assert quant_min >= lo, f"quant_min out of bound for dtype, lower bound {lo}: {quant_min}"
    assert quant_max <= hi, f"quant_max out of bound for dtype, upper bound {hi}: {quant_max}"
    return quant_min, quant_max


def _get_reduction_params(block_size, input_size):
    """Shape that exposes every quantization block as its own axis, and the block axes.

    block (1, 32) on a [4, 64] tensor -> view [4, 2, 32], reduce over [2].
    """
    assert len(block_size) == len(input_size)
    view: List[int] = []
    red: List[int] = []
    for b, s in zip(block_size, input_size):
        if b != s and b > 1:
            assert s % b == 0, f"Expecting input size {s} to be divisible by block_size {b}"
            view += [s // b, b]
            red.append(len(view) - 1)
        else:
            view.append(s)
            if b != 1:
                red.append(len(view) - 1)
    return view, red


def _qparam_view(t: torch.Tensor, block_size, input_shape):
    """Broadcastable view of per-block qparams against the reduction view of the input."""
    view, red = _get_reduction_params(block_size, input_shape)
    shape = list(view)
    for d in red:
        shape[d] = 1
    return view, t.view(shape)


class _Round(torch.autograd.Function):
    """round-half-to-even with a straight-through gradient."""

    @staticmethod
    def forward(ctx, x):
        return torch.round(x)

    @staticmethod
    def backward(ctx, gy):
        return gy


# ---------------------------------------------------------------------------------------------
# choose_qparams
# ---------------------------------------------------------------------------------------------
def _block_min_max(input: torch.Tensor, block_size):
    view, red = _get_reduction_params(block_size, input.size())
    x = input.view(view)
    return torch.amin(x, dim=red, keepdim=False), torch.amax(x, dim=red, keepdim=False)


@torch.no_grad()
def choose_qparams_affine(
    input: torch.Tensor,
    mapping_type: MappingType,
    block_size: Tuple[int, ...],
    target_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
    eps: Optional[float] = None,
    scale_dtype: Optional[torch.dtype] = None,
    zero_point_dtype: Optional[torch.dtype] = torch.int32,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-block scale / zero point preserving zero (integer zero-point domain)."""
    quant_min, quant_max = _get_and_check_qmin_qmax(target_dtype, quant_min, quant_max)
    scale_dtype = input.dtype if scale_dtype is None else scale_dtype
    eps = torch.finfo(input.dtype).eps if eps is None else eps
    assert len(block_size) == input.dim(), f"Got input dim:{input.dim()}, block_size: {block_size}"
    mn, mx = _block_min_max(input, block_size)
    mn_neg = torch.min(mn, torch.zeros_like(mn))
    mx_pos = torch.max(mx, torch.zeros_like(mx))
    if mapping_type in (MappingType.SYMMETRIC, MappingType.SYMMETRIC_NO_CLIPPING_ERR):
        if mapping_type is MappingType.SYMMETRIC:
            amax = torch.max(-mn_neg, mx_pos)
            scale = amax / (float(quant_max - quant_min) / 2)
        else:
            smin = mn_neg / float(quant_min)
            smax = mx_pos / float(quant_max)
            scale = torch.where(smin > smax, smin, smax)
        zero_point = torch.full_like(scale, int((quant_max + quant_min + 1) / 2))
        scale = torch.clamp(scale, min=eps)
    elif mapping_type is MappingType.ASYMMETRIC:
        scale = (mx_pos - mn_neg) / float(quant_max - quant_min)
        scale = torch.clamp(scale, min=eps)
        zero_point = torch.clamp(quant_min - _Round.apply(mn_neg / scale), quant_min, quant_max)
        if zero_point_dtype is None:
            zero_point_dtype = torch.int32
    else:
        raise ValueError(f"Unsupported mapping type: {mapping_type}")
    if zero_point_dtype is not None:
        zero_point = zero_point.to(dtype=zero_point_dtype)
    return scale.to(dtype=scale_dtype, device=input.device), zero_point


@torch.no_grad()
def _choose_qparams_affine_tinygemm(
    input: torch.Tensor,
    mapping_type: MappingType,
    block_size: Tuple[int, ...],
    target_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
    eps: Optional[float] = None,
    scale_dtype: Optional[torch.dtype] = None,
    zero_point_dtype: Optional[torch.dtype] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """tinygemm qparams: s = clamp((max - min) / (qmax - qmin), eps), z = min + s * mid,
    both computed in the input dtype (bf16 for Int4WeightOnlyConfig)."""
    quant_min, quant_max = _get_and_check_qmin_qmax(target_dtype, quant_min, quant_max)
    assert mapping_type is MappingType.ASYMMETRIC, f"Unsupported mapping type: {mapping_type}"
    scale_dtype = input.dtype if scale_dtype is None else scale_dtype
    eps = torch.finfo(input.dtype).eps if eps is None else eps
    assert len(block_size) == input.dim(), f"Got input dim:{input.dim()}, block_size: {block_size}"
    mn, mx = _block_min_max(input, block_size)
    scale = torch.clamp((mx - mn) / float(quant_max - quant_min), min=eps)
    mid = (quant_max + quant_min + 1) / 2
    zero_point = mn + scale * mid
    zero_point_dtype = input.dtype if zero_point_dtype is None else zero_point_dtype
    return scale.to(dtype=scale_dtype, device=input.device), zero_point.to(zero_point_dtype)


@torch.no_grad()
def _choose_qparams_affine_dont_preserve_zero(
    input: torch.Tensor,
    mapping_type: MappingType,
    block_size: Tuple[int, ...],
    target_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
    eps: Optional[float] = None,
    scale_dtype: Optional[torch.dtype] = None,
    zero_point_dtype: Optional[torch.dtype] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Integer zero-point domain WITHOUT zero preservation (quant_primitives.py:1310-1373): the
    block's own [min, max] (not widened to include 0) maps to [qmin, qmax]; s = clamp((max - min)
    / (qmax - qmin), eps), z = clamp(qmin - round(min / s), qmin, qmax) as an integer."""
    quant_min, quant_max = _get_and_check_qmin_qmax(target_dtype, quant_min, quant_max)
    assert mapping_type is MappingType.ASYMMETRIC, f"Unsupported mapping type: {mapping_type}"
    scale_dtype = input.dtype if scale_dtype is None else scale_dtype
    eps = torch.finfo(input.dtype).eps if eps is None else eps
    assert len(block_size) == input.dim(), f"Got input dim:{input.dim()}, block_size: {block_size}"
    mn, mx = _block_min_max(input, block_size)
    scale = torch.clamp((mx - mn) / float(quant_max - quant_min), min=eps)
    zero_point = torch.clamp(quant_min - _Round.apply(mn / scale), quant_min, quant_max)
    zero_point_dtype = torch.int32 if zero_point_dtype is None else zero_point_dtype
    return scale.to(dtype=scale_dtype, device=input.device), zero_point.to(dtype=zero_point_dtype)


# ---------------------------------------------------------------------------------------------
# quantize
# ---------------------------------------------------------------------------------------------
def _check_float_input(input: torch.Tensor, block_size):
    assert input.dtype in (torch.float32, torch.float16, torch.bfloat16), (
        f"Unsupported input dtype: {input.dtype}"
    )
    assert len(block_size) == input.dim(), f"Got input dim:{input.dim()}, block_size: {block_size}"


def _sub_byte_storage(dtype):
    """Sub-byte unsigned dtypes are stored in uint8 (reference quant_primitives.py:509-511)."""
    if dtype in _DTYPE_TO_QVALUE_BOUNDS and str(dtype).startswith("torch.uint") and dtype != torch.uint8:
        return torch.uint8
    return dtype


@torch.no_grad()
def quantize_affine(
    input: torch.Tensor,
    block_size: Tuple[int, ...],
    scale: torch.Tensor,
    zero_point: Optional[torch.Tensor],
    output_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
) -> torch.Tensor:
    """Integer zero-point domain: q = clamp(round(x * (1 / s)) + zp, qmin, qmax)."""
    quant_min, quant_max = _get_and_check_qmin_qmax(output_dtype, quant_min, quant_max)
    _check_float_input(input, block_size)
    view, s = _qparam_view(scale, block_size, input.shape)
    x = input.view(view)
    q = _Round.apply(x * (1.0 / s))
    if zero_point is not None and zero_point.numel() > 0:
        q = q + _qparam_view(zero_point, block_size, input.shape)[1]
    q = torch.clamp(q, quant_min, quant_max).view(input.shape)
    return q.to(_sub_byte_storage(output_dtype))


@torch.no_grad()
def _quantize_affine_no_zero_point(
    input: torch.Tensor,
    block_size: Tuple[int, ...],
    scale: torch.Tensor,
    zero_point: Optional[torch.Tensor],
    output_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
) -> torch.Tensor:
    """Zero-point-free domain: q = clamp(round(x * (1 / s)), qmin, qmax)."""
    quant_min, quant_max = _get_and_check_qmin_qmax(output_dtype, quant_min, quant_max)
    _check_float_input(input, block_size)
    view, s = _qparam_view(scale, block_size, input.shape)
    q = torch.clamp(_Round.apply(input.view(view) * (1.0 / s)), quant_min, quant_max)
    return q.view(input.shape).to(_sub_byte_storage(output_dtype))


@torch.no_grad()
def _quantize_affine_tinygemm(
    input: torch.Tensor,
    block_size: List[int],
    scale: torch.Tensor,
    zero_point: Optional[torch.Tensor],
    output_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
) -> torch.Tensor:
    """Float zero-point domain: q = clamp(round((x - (z - s * mid)) / s), qmin, qmax)."""
    quant_min, quant_max = _get_and_check_qmin_qmax(output_dtype, quant_min, quant_max)
    _check_float_input(input, block_size)
    view, s = _qparam_view(scale, block_size, input.shape)
    mid = (quant_max + quant_min + 1) / 2
    if zero_point is not None and zero_point.numel() > 0:
        z = _qparam_view(zero_point, block_size, input.shape)[1]
        lo = z - s * mid
        q = _Round.apply((input.view(view) - lo) / s)
    else:
        q = _Round.apply(input.view(view) / s)
    q = torch.clamp(q, quant_min, quant_max).view(input.shape)
    return q.to(_sub_byte_storage(output_dtype))


# ---------------------------------------------------------------------------------------------
# dequantize
# ---------------------------------------------------------------------------------------------
@torch.no_grad()
def dequantize_affine(
    input: torch.Tensor,
    block_size: Tuple[int, ...],
    scale: torch.Tensor,
    zero_point: Optional[torch.Tensor],
    input_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
    *,
    output_dtype: torch.dtype = torch.float32,
) -> torch.Tensor:
    """Integer zero-point domain: x = (q - zp) * s, evaluated in ``output_dtype``."""
    _get_and_check_qmin_qmax(input_dtype, quant_min, quant_max)
    view, s = _qparam_view(scale, block_size, input.shape)
    x = input.view(view).to(output_dtype, copy=True)
    if zero_point is not None:
        x = x - _qparam_view(zero_point, block_size, input.shape)[1].to(output_dtype)
    x = x * s
    return x.view(input.shape).to(output_dtype)


@torch.no_grad()
def _dequantize_affine_no_zero_point(
    input: torch.Tensor,
    block_size: Tuple[int, ...],
    scale: torch.Tensor,
    zero_point: Optional[torch.Tensor],
    input_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
    *,
    output_dtype: torch.dtype = torch.float32,
) -> torch.Tensor:
    """x = q * s."""
    _get_and_check_qmin_qmax(input_dtype, quant_min, quant_max)
    view, s = _qparam_view(scale, block_size, input.shape)
    x = input.view(view).to(output_dtype, copy=True) * s
    return x.view(input.shape).to(output_dtype)


@torch.no_grad()
def _dequantize_affine_tinygemm(
    input: torch.Tensor,
    block_size: Tuple[int, ...],
    scale: torch.Tensor,
    zero_point: Optional[torch.Tensor],
    input_dtype: torch.dtype,
    quant_min: Optional[Union[int, float]] = None,
    quant_max: Optional[Union[int, float]] = None,
    *,
    output_dtype: torch.dtype = torch.float32,
) -> torch.Tensor:
    """Float zero-point domain: x = (q - mid).to(out) * s + z — two roundings in ``output_dtype``
    (the multiply, then the add), as the reference (quant_primitives.py:1017-1023)."""
    quant_min, quant_max = _get_and_check_qmin_qmax(input_dtype, quant_min, quant_max)
    view, s = _qparam_view(scale, block_size, input.shape)
    mid = (quant_max + quant_min + 1) / 2
    x = (input.view(view) - mid).to(output_dtype)
    x *= s  # in place: stays in output_dtype, one rounding
    if zero_point is not None:
        x += _qparam_view(zero_point, block_size, input.shape)[1]  # second rounding
    return x.view(input.shape).to(output_dtype)


# enums appear in flattened AQT metadata: allow weights_only=True checkpoint loads
torch.serialization.add_safe_globals([MappingType, ZeroPointDomain])
