"""Plain (int_data, scale, zero_point) layout and the int8 linear impls on MI355X.

Reference: torchao/dtypes/uintx/plain_layout.py. ``PlainAQTTensorImpl`` (:48-212) stores the
quantized tensors as they are. Two quantized-linear pairs are registered from here:

* int8 weight-only (:232-266): the reference runs ``torch.mm(x, w.t().to(x.dtype)) * scale``,
  materialising a bf16 copy of W; here ``torch.ops.torchao.int8_weight_only_linear`` reads the
  int8 weight once (HIP GEMV for M <= 2, or M <= 4 for weights of at most 32 Mi elements;
  bf16-MFMA tiles above) with the same three bf16
  roundings (mm output, * scale, + bias).
* int8 dynamic activation x int8 weight (:269-315): ``int_scaled_matmul`` + weight scale become
  one int8-MFMA kernel with the two scales fused in its epilogue
  (``torch.ops.torchao.int8_scaled_mm``).

Both HIP impls take bf16 activations (the dtype of the hot path); other activation dtypes do not
match the checks and take the table's generic dequantize -> F.linear route, as any unmatched
input does in the reference.
"""

from typing import Optional, Tuple

import torch
from torch.utils._python_dispatch import (
    is_traceable_wrapper_subclass,
    return_and_correct_aliasing,
)

from torchao.dtypes.affine_quantized_tensor import AffineQuantizedTensor, register_layout
from torchao.dtypes.utils import AQTTensorImpl, Layout, PlainLayout
from torchao.quantization.quant_primitives import ZeroPointDomain
from torchao.utils import fill_defaults

aten = torch.ops.aten

__all__ = ["PlainAQTTensorImpl"]


@register_layout(PlainLayout)
class PlainAQTTensorImpl(AQTTensorImpl):
    """``int_data`` / ``scale`` / ``zero_point`` kept as plain tensors."""

    def __new__(cls, int_data, scale, zero_point, _layout):
        return torch.Tensor._make_wrapper_subclass(
            cls,
            int_data.shape,
            device=int_data.device,
            layout=int_data.layout,
            dtype=int_data.dtype,
            requires_grad=False,
        )

    def __init__(
        self,
        int_data: torch.Tensor,
        scale: torch.Tensor,
        zero_point: Optional[torch.Tensor],
        _layout: Layout,
    ):
        self.int_data = int_data
        self.scale = scale
        self.zero_point = zero_point
        self._layout = _layout

    def __tensor_flatten__(self):
        names = ["int_data", "scale"] + ([] if self.zero_point is None else ["zero_point"])
        return names, [self._layout]

    @classmethod
    def __tensor_unflatten__(cls, tensor_data_dict, tensor_attributes, outer_size, outer_stride):
        (layout,) = tensor_attributes
        return cls(
            tensor_data_dict["int_data"],
            tensor_data_dict["scale"],
            tensor_data_dict.get("zero_point", None),
            layout,
        )

    def to(self, *args, **kwargs):
        device = self._get_to_kwargs(*args, **kwargs)["device"]
        return type(self)(
            self.int_data.to(device),
            self.scale.to(device),
            None if self.zero_point is None else self.zero_point.to(device),
            self._layout,
        )

    def _apply_fn_to_data(self, fn):
        return type(self)(
            fn(self.int_data),
            fn(self.scale),
            None if self.zero_point is None else fn(self.zero_point),
            self._layout,
        )

    @classmethod
    def __torch_dispatch__(cls, func, types, args, kwargs):
        kwargs = {} if kwargs is None else kwargs
        if func is aten.detach.default:
            return return_and_correct_aliasing(
                func, args, kwargs, args[0]._apply_fn_to_data(torch.detach)
            )
        if func is aten.clone.default:
            return return_and_correct_aliasing(
                func, args, kwargs, args[0]._apply_fn_to_data(torch.clone)
            )
        if func is aten.copy_.default:
            dst, src = args[0], args[1]
            if (
                isinstance(src, cls)
                and dst.int_data.shape == src.int_data.shape
                and dst.scale.shape == src.scale.shape
                and (dst.zero_point is None) == (src.zero_point is None)
                and (dst.zero_point is None or dst.zero_point.shape == src.zero_point.shape)
                and type(dst._layout) is type(src._layout)
            ):
                for name in dst.__tensor_flatten__()[0]:
                    getattr(dst, name).copy_(getattr(src, name))
                return
            raise ValueError(f"Not supported args for copy_ due to metadata mismatch: {dst, src}")
        if func is aten.t.default:
            t = args[0]
            new = cls(t.int_data.t(), t.scale, t.zero_point, t._layout)
            return return_and_correct_aliasing(func, args, kwargs, new)
        if func in (aten.select.int, aten.index.Tensor):
            return return_and_correct_aliasing(
                func,
                args,
                kwargs,
                args[0]._apply_fn_to_data(lambda t: func(t, *args[1:], **kwargs)),
            )
        if func is aten.slice.Tensor:
            self, dim, start, end, step = fill_defaults(args, 5, [0, None, None, 1])
            if dim == 0:
                return return_and_correct_aliasing(
                    func,
                    args,
                    kwargs,
                    self._apply_fn_to_data(lambda t: aten.slice.Tensor(t, dim, start, end, step)),
                )
            if dim == 1:
                assert self.scale.dim() == 1 or self.scale.shape[-1] == 1, (
                    f"slice dim==1 needs per-row scales, got {self.scale.shape}"
                )
                return cls(
                    aten.slice.Tensor(self.int_data, dim, start, end, step),
                    self.scale.view(-1),
                    None if self.zero_point is None else self.zero_point.view(-1),
                    self._layout,
                )
            raise NotImplementedError(f"PlainAQTTensorImpl: slice on dim {dim} is not supported")
        raise NotImplementedError(f"PlainAQTTensorImpl dispatch: {func} is not supported")

    __torch_function__ = torch._C._disabled_torch_function_impl

    def get_plain(self) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
        return self.int_data, self.scale, self.zero_point

    def get_layout(self) -> Layout:
        return self._layout

    @classmethod
    def from_plain(cls, int_data, scale, zero_point, _layout):
        assert isinstance(_layout, PlainLayout)
        return cls(int_data, scale, zero_point, _layout)


def _aqt_is_int8(aqt) -> bool:
    return (
        aqt.tensor_impl.dtype == torch.int8
        and (aqt.quant_min is None or aqt.quant_min == -128)
        and (aqt.quant_max is None or aqt.quant_max == 127)
    )


def _aqt_is_int8_reduced_range(aqt) -> bool:
    return (
        aqt.tensor_impl.dtype == torch.int8
        and aqt.quant_min == -127
        and (aqt.quant_max is None or aqt.quant_max == 127)
    )


def _linear_fp_act_int8_weight_check(input_tensor, weight_tensor, bias) -> bool:
    return (
        not is_traceable_wrapper_subclass(input_tensor)
        and input_tensor.dtype == torch.bfloat16
        and isinstance(weight_tensor, AffineQuantizedTensor)
        and _aqt_is_int8(weight_tensor)
        and len(weight_tensor.shape) == 2
        and len(weight_tensor.block_size) == 2
        and weight_tensor.block_size[0] == 1
        and weight_tensor.block_size[1] == weight_tensor.shape[1]
        and weight_tensor.zero_point_domain == ZeroPointDomain.INT
        and isinstance(weight_tensor._layout, PlainLayout)
    )


def _linear_fp_act_int8_weight_impl(input_tensor, weight_tensor, bias):
    """y = bf16(bf16(x @ W^T) * scale) (+ bias), W int8 per-channel (reference :250-266)."""
    impl = weight_tensor.tensor_impl
    return torch.ops.torchao.int8_weight_only_linear(
        input_tensor, impl.int_data, impl.scale.reshape(-1), bias
    )


def _linear_int8_act_int8_weight_check(input_tensor, weight_tensor, bias) -> bool:
    return (
        isinstance(input_tensor, AffineQuantizedTensor)
        and _aqt_is_int8_reduced_range(input_tensor)
        and isinstance(weight_tensor, AffineQuantizedTensor)
        and _aqt_is_int8(weight_tensor)
        and input_tensor.dtype == weight_tensor.dtype
        and input_tensor.dtype == torch.bfloat16
        and isinstance(input_tensor._layout, PlainLayout)
        and isinstance(weight_tensor._layout, PlainLayout)
    )


def _linear_int8_act_int8_weight_impl(input_tensor, weight_tensor, bias):
    """y = bf16(bf16(float(xq @ wq^T) * s_x) * s_w) (+ bias) (reference :281-315)."""
    x_impl = input_tensor.tensor_impl
    w_impl = weight_tensor.tensor_impl
    y = torch.ops.torchao.int8_scaled_mm(
        x_impl.int_data,
        x_impl.scale,
        w_impl.int_data,
        w_impl.scale.reshape(-1),
        bias,
    )
    return y.to(input_tensor.dtype)
