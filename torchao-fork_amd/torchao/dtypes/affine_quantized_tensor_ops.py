"""Operator overrides of ``AffineQuantizedTensor`` and the quantized-linear plug-in table.

Reference: torchao/dtypes/affine_quantized_tensor_ops.py. The plug-in point is an ordered table
of ``(dispatch_condition, impl)`` pairs (:113-139); the first condition that accepts
``(input, weight, bias)`` runs its impl (:172-183). ``F.linear`` / ``aten.addmm`` / ``aten.mm``
route through it (:267-419) and fall back to ``dequantize() -> F.linear`` when nothing matches
and the layout does not insist on its own impl. The aten view / copy ops (:422-598) keep the
subclass usable inside ``nn.Linear``, ``DTensor.from_local`` and state-dict loading.

The pairs registered here are the MI355X ones, in the reference's order of precedence:
int8 dynamic-activation x int8 weight, int8 weight-only, int4 weight-only (gfx950 layout).
"""

import logging

import torch
from torch.utils._python_dispatch import return_and_correct_aliasing

from torchao.dtypes.affine_quantized_tensor import AffineQuantizedTensor
from torchao.dtypes.uintx.plain_layout import (
    _linear_fp_act_int8_weight_check,
    _linear_fp_act_int8_weight_impl,
    _linear_int8_act_int8_weight_check,
    _linear_int8_act_int8_weight_impl,
)
from torchao.dtypes.uintx.tensor_core_tiled_layout import (
    _linear_bf16_act_uint4_weight_check,
    _linear_bf16_act_uint4_weight_impl,
)
from torchao.utils import fill_defaults

logger = logging.getLogger(__name__)
aten = torch.ops.aten

_AQT_QLINEAR_DISPATCH_TABLE = {}


def register_aqt_quantized_linear_dispatch(dispatch_condition, impl):
    """Add a specialised quantized-linear implementation: ``dispatch_condition(x, w, bias)``
    decides, ``impl(x, w, bias)`` computes. x: (..., in_features), w: (out, in), bias: (out,)."""
    _AQT_QLINEAR_DISPATCH_TABLE[dispatch_condition] = impl


def deregister_aqt_quantized_linear_dispatch(dispatch_condition):
    if dispatch_condition in _AQT_QLINEAR_DISPATCH_TABLE:
        del _AQT_QLINEAR_DISPATCH_TABLE[dispatch_condition]
    else:
        logger.warning(
            f"Attempting to remove non-existent dispatch condition {dispatch_condition}"
        )


class QuantizedLinearNotImplementedError(NotImplementedError):
    """No entry of the dispatch table accepted the arguments."""


def _quantized_linear_op(input_tensor, weight_tensor, bias):
    for condition, impl in _AQT_QLINEAR_DISPATCH_TABLE.items():
        if condition(input_tensor, weight_tensor, bias):
            return impl(input_tensor, weight_tensor, bias)
    raise QuantizedLinearNotImplementedError(
        "No specialized dispatch found for quantized linear op"
    )


AffineQuantizedTensor._quantized_linear_op = staticmethod(_quantized_linear_op)

for _cond, _impl in [
    (_linear_int8_act_int8_weight_check, _linear_int8_act_int8_weight_impl),
    (_linear_fp_act_int8_weight_check, _linear_fp_act_int8_weight_impl),
    (_linear_bf16_act_uint4_weight_check, _linear_bf16_act_uint4_weight_impl),
]:
    register_aqt_quantized_linear_dispatch(_cond, _impl)

implements = AffineQuantizedTensor.implements


def _insists_on_own_impl(weight_tensor) -> bool:
    return (
        isinstance(weight_tensor, AffineQuantizedTensor)
        and getattr(weight_tensor._layout, "quantized_linear_impl", None) is not None
    )


def _dequantized(t):
    return t.dequantize() if isinstance(t, AffineQuantizedTensor) else t


@implements([torch.nn.functional.linear, aten.linear.default])
def _(func, types, args, kwargs):
    input_tensor = args[0]
    weight_tensor = args[1]
    bias = args[2] if len(args) > 2 else kwargs.get("bias", None)
    if not input_tensor.is_floating_point():
        raise NotImplementedError(f"{func} is not implemented for non floating point input")
    try:
        return weight_tensor._quantized_linear_op(input_tensor, weight_tensor, bias)
    except QuantizedLinearNotImplementedError:
        if _insists_on_own_impl(weight_tensor):
            raise
        return torch.nn.functional.linear(
            _dequantized(input_tensor), _dequantized(weight_tensor), bias
        )


@implements(aten.addmm.default)
def _(func, types, args, kwargs):
    bias, input_tensor, weight_tensor = args[0], args[1], args[2]
    if not input_tensor.is_floating_point():
        raise NotImplementedError(f"{func} is not implemented for non floating point input")
    assert input_tensor.shape[-1] == weight_tensor.shape[0], (
        f"need mat1 shape: {input_tensor.shape} final dim"
        f"to match mat2 shape: {weight_tensor.shape} first dim"
    )
    try:
        return weight_tensor._quantized_linear_op(input_tensor, weight_tensor.t(), bias)
    except QuantizedLinearNotImplementedError:
        if _insists_on_own_impl(weight_tensor):
            raise
        return func(bias, _dequantized(input_tensor), _dequantized(weight_tensor))


@implements(aten.mm.default)
def _(func, types, args, kwargs):
    input_tensor, weight_tensor = args[0], args[1]
    if not input_tensor.is_floating_point():
        raise NotImplementedError(f"{func} is not implemented for non floating point input")
    assert input_tensor.shape[-1] == weight_tensor.shape[0], (
        f"need mat1 shape: {input_tensor.shape} final dim"
        f"to match mat2 shape: {weight_tensor.shape} first dim"
    )
    try:
        return weight_tensor._quantized_linear_op(input_tensor, weight_tensor.t(), None)
    except QuantizedLinearNotImplementedError:
        if _insists_on_own_impl(weight_tensor):
            raise
        return func(_dequantized(input_tensor), _dequantized(weight_tensor))


@implements([aten.detach.default, aten.alias.default])
def _(func, types, args, kwargs):
    return return_and_correct_aliasing(
        func, args, kwargs, args[0]._apply_fn_to_data(torch.detach)
    )


@implements(aten.clone.default)
def _(func, types, args, kwargs):
    return return_and_correct_aliasing(
        func, args, kwargs, args[0]._apply_fn_to_data(torch.clone)
    )


@implements(aten._to_copy.default)
def _(func, types, args, kwargs):
    return return_and_correct_aliasing(
        func, args, kwargs, args[0].to(*args[1:], **kwargs)._apply_fn_to_data(torch.clone)
    )


def _same_metadata(a, b) -> bool:
    attrs = ("block_size", "shape", "quant_min", "quant_max", "zero_point_domain", "dtype")
    return (
        isinstance(a, AffineQuantizedTensor)
        and isinstance(b, AffineQuantizedTensor)
        and all(getattr(a, n) == getattr(b, n) for n in attrs)
        and isinstance(a.tensor_impl, type(b.tensor_impl))
    )


@implements(aten.copy_.default)
def _(func, types, args, kwargs):
    dst, src = args[0], args[1]
    if _same_metadata(dst, src):
        for name in dst.__tensor_flatten__()[0]:
            getattr(dst, name).copy_(getattr(src, name))
        return
    raise ValueError(f"Not supported args for copy_ due to metadata mismatch: {dst, src}")


@implements(aten.t.default)
def _(func, types, args, kwargs):
    t = args[0]
    assert len(t.block_size) == 2
    new = type(t)(
        t.tensor_impl.t(),
        (t.block_size[1], t.block_size[0]),
        t.shape[::-1],
        t.quant_min,
        t.quant_max,
        t.zero_point_domain,
        dtype=t.dtype,
        strides=t.stride(),
    )
    return return_and_correct_aliasing(func, args, kwargs, new)


@implements(aten.slice.Tensor)
def _(func, types, args, kwargs):
    self, dim, start, end, step = fill_defaults(args, 5, [0, None, None, 1])
    assert step == 1, "only step 1 slicing is supported"
    assert dim in (0, 1), f"Only dim==0 or 1 are supported, got: {dim}"
    start = 0 if start is None else start
    end = self.shape[dim] if end is None else min(end, self.shape[dim])
    shape = list(self.shape)
    shape[dim] = end - start
    block_size = self.block_size
    assert len(block_size) in (2, 3), f"Slice needs a 2d/3d block_size, got: {block_size}"
    if len(block_size) == 2:
        block_size = (min(shape[0], block_size[0]), min(shape[1], block_size[1]))
    new = type(self)(
        aten.slice.Tensor(self.tensor_impl, dim, start, end, step),
        block_size,
        shape,
        self.quant_min,
        self.quant_max,
        self.zero_point_domain,
        dtype=self.dtype,
        strides=self.stride() if len(block_size) == 2 else None,
    )
    return return_and_correct_aliasing(func, args, kwargs, new)


@implements(aten.index.Tensor)
def _(func, types, args, kwargs):
    self, indices = args
    assert len(indices) == 1, "only single-dimension indexing is supported"
    new = type(self)(
        aten.index.Tensor(self.tensor_impl, indices),
        self.block_size,
        (indices[0].numel(), *self.shape[1:]),
        self.quant_min,
        self.quant_max,
        self.zero_point_domain,
        dtype=self.dtype,
    )
    return return_and_correct_aliasing(func, args, kwargs, new)


@implements(aten.select.int)
def _(func, types, args, kwargs):
    self, dim, index = fill_defaults(args, 3, [0, 0])
    assert dim == 0 and self.dim() == 3, "select is supported on dim 0 of 3d tensors"
    new = type(self)(
        aten.select.int(self.tensor_impl, dim, index),
        self.block_size[1:],
        self.shape[1:],
        self.quant_min,
        self.quant_max,
        self.zero_point_domain,
        dtype=self.dtype,
    )
    return return_and_correct_aliasing(func, args, kwargs, new)


@implements(aten.view.default)
def _(func, types, args, kwargs):
    self, shape = args
    if tuple(self.shape) == tuple(shape):
        return type(self)(
            self.tensor_impl,
            self.block_size,
            self.shape,
            self.quant_min,
            self.quant_max,
            self.zero_point_domain,
            dtype=self.dtype,
            strides=self.stride(),
        )
    if len(shape) == 1 and shape[0] == -1:
        assert len(self.block_size) == 2 and self.block_size[0] == 1
        return type(self)(
            self.tensor_impl,
            (self.block_size[1],),
            (self.numel(),),
            self.quant_min,
            self.quant_max,
            self.zero_point_domain,
            dtype=self.dtype,
            strides=self.stride(),
        )
    raise ValueError(f"{type(self).__name__} only supports .view() with same shape or shape=[-1]")
