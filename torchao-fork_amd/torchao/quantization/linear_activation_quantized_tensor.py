"""``LinearActivationQuantizedTensor`` — dynamic activation quantization wrapper.

Reference: torchao/quantization/linear_activation_quantized_tensor.py:21-288. The weight is an
(already quantized) tensor; on ``F.linear`` the activation goes through ``input_quant_func``
first and the pair dispatches again (into the AQT table, e.g. the int8 x int8 MFMA impl).
"""

from typing import Any, Callable, Dict, Optional

import torch
from torch.utils._python_dispatch import return_and_correct_aliasing

from torchao.utils import TorchAOBaseTensor

__all__ = ["LinearActivationQuantizedTensor", "to_linear_activation_quantized"]

aten = torch.ops.aten


class LinearActivationQuantizedTensor(TorchAOBaseTensor):
    """Weight wrapper that quantizes the linear's input with ``input_quant_func``."""

    quant_kwargs: Dict[str, Any]

    def __new__(cls, original_weight_tensor, input_quant_func, quant_kwargs):
        return torch.Tensor._make_wrapper_subclass(
            cls,
            original_weight_tensor.shape,
            dtype=original_weight_tensor.dtype,
            device=original_weight_tensor.device,
            requires_grad=False,
        )

    def __init__(
        self,
        original_weight_tensor: torch.Tensor,
        input_quant_func: Callable[[torch.Tensor], torch.Tensor],
        quant_kwargs: Dict[str, Any],
    ):
        self.original_weight_tensor = original_weight_tensor
        self.input_quant_func = input_quant_func
        self.quant_kwargs = quant_kwargs

    def __repr__(self):
        return (
            f"{type(self).__name__}({self.original_weight_tensor}, {self.input_quant_func}, "
            f"quant_kwargs={self.quant_kwargs}))"
        )

    def __tensor_flatten__(self):
        return ["original_weight_tensor"], [self.input_quant_func, self.quant_kwargs]

    @classmethod
    def __tensor_unflatten__(cls, tensor_data_dict, tensor_attributes, outer_size, outer_stride):
        input_quant_func, quant_kwargs = tensor_attributes
        return cls(tensor_data_dict["original_weight_tensor"], input_quant_func, quant_kwargs)

    @staticmethod
    def _quantized_linear_op(input_tensor, weight_tensor, bias):
        if input_tensor.numel() == 0:
            return input_tensor
        y = _fused_int8_dyn_decode(input_tensor, weight_tensor, bias)
        if y is not None:
            return y
        qx = weight_tensor.input_quant_func(input_tensor, **weight_tensor.quant_kwargs)
        return torch.nn.functional.linear(qx, weight_tensor.original_weight_tensor, bias)

    @classmethod
    def from_float(
        cls,
        input_float: torch.Tensor,
        input_quant_func: Callable,
        quant_kwargs: Optional[Dict[str, Any]] = None,
    ):
        return cls(input_float, input_quant_func, {} if quant_kwargs is None else quant_kwargs)

    def _apply_fn_to_data(self, fn):
        return type(self)(fn(self.original_weight_tensor), self.input_quant_func, self.quant_kwargs)

    def to(self, *args, **kwargs):
        kwargs = self._get_to_kwargs(*args, **kwargs)
        return type(self)(
            self.original_weight_tensor.to(**kwargs), self.input_quant_func, self.quant_kwargs
        )


def _fused_int8_dyn_decode(x, weight_tensor, bias):
    """One bf16 token on the GPU with the default Int8DynamicActivationInt8WeightConfig recipe
    (per-token reduced-range quant, plain int8 per-channel weight): quantise + int8 GEMV in one
    launch (``torch.ops.torchao.int8_dyn_linear``), bit-identical to quantising the input and
    dispatching F.linear(AQT x, AQT w) to ``_linear_int8_act_int8_weight_impl``. Any other
    recipe, shape or device returns None and takes the reference path above."""
    from torchao.dtypes.affine_quantized_tensor import AffineQuantizedTensor
    from torchao.dtypes.uintx.plain_layout import PlainLayout, _aqt_is_int8
    from torchao.quantization.quant_api import _int8_symm_per_token_reduced_range_quant

    if weight_tensor.input_quant_func is not _int8_symm_per_token_reduced_range_quant:
        return None
    if weight_tensor.quant_kwargs or not isinstance(x, torch.Tensor) or type(x) is not torch.Tensor:
        return None
    K = x.shape[-1]
    if not (x.is_cuda and x.dtype == torch.bfloat16 and K % 16 == 0 and x.numel() == K):
        return None
    w = weight_tensor.original_weight_tensor
    if not (isinstance(w, AffineQuantizedTensor) and _aqt_is_int8(w) and w.dtype == torch.bfloat16
            and isinstance(w._layout, PlainLayout) and len(w.shape) == 2 and w.shape[1] == K
            and w.tensor_impl.int_data.is_cuda):
        return None
    impl = w.tensor_impl
    return torch.ops.torchao.int8_dyn_linear(x, impl.int_data, impl.scale.reshape(-1), bias)


implements = LinearActivationQuantizedTensor.implements


@implements([torch.nn.functional.linear, aten.linear.default])
def _(func, types, args, kwargs):
    input_tensor, weight_tensor = args[0], args[1]
    bias = args[2] if len(args) > 2 else kwargs.get("bias", None)
    if isinstance(weight_tensor, LinearActivationQuantizedTensor):
        return weight_tensor._quantized_linear_op(input_tensor, weight_tensor, bias)
    raise NotImplementedError(
        "LinearActivationQuantizedTensor: No specialized dispatch found for linear op"
    )


@implements([aten.mm.default, aten.addmm.default])
def _(func, types, args, kwargs):
    if not args[0].is_floating_point():
        raise NotImplementedError("LinearActivationQuantizedTensor: expecting a floating point input")
    if func == aten.addmm.default:
        bias, x, w = args[0], args[1], args[2]
        return func(bias, w.input_quant_func(x, **w.quant_kwargs), w.original_weight_tensor)
    x, w = args[0], args[1]
    return func(w.input_quant_func(x, **w.quant_kwargs), w.original_weight_tensor)


@implements([aten.detach.default, aten.alias.default])
def _(func, types, args, kwargs):
    return return_and_correct_aliasing(func, args, kwargs, args[0]._apply_fn_to_data(func))


@implements(aten.clone.default)
def _(func, types, args, kwargs):
    return return_and_correct_aliasing(func, args, kwargs, args[0]._apply_fn_to_data(torch.clone))


@implements(aten._to_copy.default)
def _(func, types, args, kwargs):
    return return_and_correct_aliasing(
        func, args, kwargs, args[0].to(*args[1:], **kwargs)._apply_fn_to_data(torch.clone)
    )


@implements(aten.copy_.default)
def _(func, types, args, kwargs):
    dst, src = args[0], args[1]
    if (
        isinstance(dst, LinearActivationQuantizedTensor)
        and isinstance(src, LinearActivationQuantizedTensor)
        and dst.shape == src.shape
        and dst.input_quant_func == src.input_quant_func
        and dst.quant_kwargs == src.quant_kwargs
    ):
        dst.original_weight_tensor.copy_(src.original_weight_tensor)
        return
    raise ValueError(f"Not supported args for copy_ due to metadata mismatch: {dst, src}")


@implements(aten.t.default)
def _(func, types, args, kwargs):
    return return_and_correct_aliasing(func, args, kwargs, args[0]._apply_fn_to_data(torch.t))


@implements([aten.slice.Tensor, aten.select.int, aten.index.Tensor, aten.view.default])
def _(func, types, args, kwargs):
    w = args[0]
    return return_and_correct_aliasing(
        func,
        args,
        kwargs,
        LinearActivationQuantizedTensor(
            func(w.original_weight_tensor, *args[1:]), w.input_quant_func, w.quant_kwargs
        ),
    )


to_linear_activation_quantized = LinearActivationQuantizedTensor.from_float

torch.serialization.add_safe_globals([LinearActivationQuantizedTensor])
