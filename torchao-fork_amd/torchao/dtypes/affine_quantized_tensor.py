"""``AffineQuantizedTensor`` — the quantized-weight tensor subclass.

Mirrors the reference (torchao/dtypes/affine_quantized_tensor.py:57-614) for the integer
workflows on the hot path: ``from_hp_to_intx`` (pre_process -> choose_qparams -> quantize ->
post_process -> layout constructor, :231-373), ``from_hp_to_intx_static``, ``dequantize``
(:134-196), flatten/unflatten (:198-229), ``to`` and ``_apply_fn_to_data``. The float8 /
floatx / HQQ constructors belong to out-of-scope workflows and are not provided.
"""

import logging
from typing import Optional, Tuple, Union

import torch

from torchao.dtypes.utils import AQTTensorImpl, Layout, PlainLayout
from torchao.quantization.quant_primitives import (
    MappingType,
    ZeroPointDomain,
    _choose_qparams_affine_tinygemm,
    _dequantize_affine_no_zero_point,
    _dequantize_affine_tinygemm,
    _quantize_affine_no_zero_point,
    _quantize_affine_tinygemm,
    choose_qparams_affine,
    dequantize_affine,
    quantize_affine,
)
from torchao.utils import TorchAOBaseTensor

logger = logging.getLogger(__name__)
aten = torch.ops.aten

__all__ = [
    "AffineQuantizedTensor",
    "register_layout",
    "to_affine_quantized_intx",
    "to_affine_quantized_intx_static",
]


def _fused_weight_quant(x, mapping_type, block_size, target_dtype, quant_min, quant_max, eps,
                        scale_dtype, zero_point_dtype, preserve_zero, zero_point_domain, layout):
    """The tensor impl from one fused gfx950 quantizer kernel, or None to take the torch-op
    path. Covers the two weight recipes of the hot path on bf16 CUDA weights, with results
    bit-identical to the torch-op path (tests/test_gpu_quantize.py):
      * int4 tinygemm (Int4WeightOnlyConfig): ASYMMETRIC, FLOAT zero domain, preserve_zero
        False, [0, 15], blocks (1, ..., g) -> torchao::int4_quantize_pack straight into the
        TensorCoreTiledLayout impl (no int32 [N, K] intermediate, no separate pack);
      * int8 symmetric per row (Int8WeightOnlyConfig, int8 dyn weights): SYMMETRIC, blocks
        (1, ..., K), [-128, 127] -> torchao::int8_quantize_rows into the PlainLayout impl."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() in (2, 3) and eps is not None):
        return None
    if any(b != 1 for b in block_size[:-1]):
        return None
    K = x.shape[-1]
    g = block_size[-1]
    from torchao.dtypes.uintx.tensor_core_tiled_layout import (
        TensorCoreTiledAQTTensorImpl,
        TensorCoreTiledLayout,
    )

    if (
        isinstance(layout, TensorCoreTiledLayout)
        and mapping_type is MappingType.ASYMMETRIC
        and zero_point_domain == ZeroPointDomain.FLOAT
        and not preserve_zero
        and target_dtype == torch.int32
        and (quant_min, quant_max) == (0, 15)
        and g in (32, 64, 128, 256)
        and K % g == 0
        and scale_dtype in (None, torch.bfloat16)
        and zero_point_dtype in (None, torch.bfloat16)
    ):
        packed, sz = torch.ops.torchao.int4_quantize_pack(x, g, float(eps))
        return TensorCoreTiledAQTTensorImpl(packed, sz, False, layout)
    if (
        type(layout) is PlainLayout
        and mapping_type is MappingType.SYMMETRIC
        and zero_point_domain in (ZeroPointDomain.INT, ZeroPointDomain.NONE)
        and preserve_zero
        and target_dtype == torch.int8
        and quant_min in (None, -128)
        and quant_max in (None, 127)
        and g == K
        and K % 8 == 0
        and scale_dtype in (None, torch.bfloat16)
    ):
        q, scale = torch.ops.torchao.int8_quantize_rows(x, float(eps))
        zero_point = None
        if zero_point_domain == ZeroPointDomain.INT:
            zero_point = torch.zeros_like(scale, dtype=zero_point_dtype or torch.int32)
        q, scale, zero_point = layout.post_process(q, scale, zero_point, block_size)
        return AffineQuantizedTensor.get_tensor_impl_constructor(type(layout))(
            q, scale, zero_point, layout
        )
    return None


def _adopt_loaded_impl(impl, shape):
    """A layout impl may recognise storage written by another build and convert it
    (``_adopt(shape)``, e.g. the reference's int4 tile format); others pass through."""
    adopt = getattr(type(impl), "_adopt", None)
    return impl if adopt is None else adopt(impl, tuple(shape))


class AffineQuantizedTensor(TorchAOBaseTensor):
    """float_tensor ~= dequantize(tensor_impl) with qparams shared over ``block_size`` blocks.

    fields: ``tensor_impl`` (layout-specific storage), ``block_size``, ``shape`` (of the
    original high-precision tensor), ``quant_min`` / ``quant_max``, ``zero_point_domain``,
    ``dtype`` (of the original high-precision tensor).
    """

    @staticmethod
    def __new__(
        cls,
        tensor_impl: AQTTensorImpl,
        block_size: Tuple[int, ...],
        shape: torch.Size,
        quant_min: Optional[Union[int, float]] = None,
        quant_max: Optional[Union[int, float]] = None,
        zero_point_domain: ZeroPointDomain = ZeroPointDomain.INT,
        dtype=None,
        strides=None,
    ):
        if zero_point_domain is None:
            raise ValueError("please use ZeroPointDomain.NONE instead of None")
        kwargs = {
            "device": tensor_impl.device,
            "layout": tensor_impl.layout,
            "dtype": dtype,
            "requires_grad": False,
        }
        if strides is not None:
            kwargs["strides"] = strides
        return torch.Tensor._make_wrapper_subclass(cls, shape, **kwargs)

    def __init__(
        self,
        tensor_impl: AQTTensorImpl,
        block_size: Tuple[int, ...],
        shape: torch.Size,
        quant_min: Optional[Union[int, float]] = None,
        quant_max: Optional[Union[int, float]] = None,
        zero_point_domain: ZeroPointDomain = ZeroPointDomain.INT,
        dtype=None,
        strides=None,
    ):
        self.tensor_impl = tensor_impl
        self.block_size = block_size
        self.quant_min = quant_min
        self.quant_max = quant_max
        self.zero_point_domain = zero_point_domain

    def __repr__(self):
        return (
            f"{type(self).__name__}(tensor_impl={self.tensor_impl}, block_size={self.block_size}, "
            f"shape={self.shape}, device={self.device}, dtype={self.dtype}, "
            f"requires_grad={self.requires_grad})"
        )

    def _quantization_type(self):
        return (
            f"shape={self.shape}, block_size={self.block_size}, device={self.device}, "
            f"_layout={self._layout}, tensor_impl_dtype={self.tensor_impl.dtype}, "
            f"quant_min={self.quant_min}, quant_max={self.quant_max}"
        )

    @property
    def _layout(self) -> Layout:
        return self.tensor_impl._layout

    def dequantize(self, output_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """High-precision tensor of ``self.shape``: get_plain() -> the domain's dequant formula."""
        output_dtype = self.dtype if output_dtype is None else output_dtype
        data, scale, zero_point = self.tensor_impl.get_plain()
        if self.zero_point_domain == ZeroPointDomain.FLOAT:
            fn = _dequantize_affine_tinygemm
        elif self.zero_point_domain == ZeroPointDomain.NONE:
            fn = _dequantize_affine_no_zero_point
        else:
            fn = dequantize_affine
        dq = fn(
            data,
            self.block_size,
            scale,
            zero_point,
            data.dtype,
            self.quant_min,
            self.quant_max,
            output_dtype=output_dtype,
        )
        # layouts may pad; return the logical shape
        for dim, size in enumerate(self.shape):
            if dq.shape[dim] != size:
                dq = dq.narrow(dim, 0, size)
        return dq

    def __tensor_flatten__(self):
        with torch._C.DisableTorchFunctionSubclass():
            return ["tensor_impl"], [
                self.block_size,
                self.shape,
                self.quant_min,
                self.quant_max,
                self.zero_point_domain,
                self.dtype,
            ]

    @classmethod
    def __tensor_unflatten__(cls, tensor_data_dict, tensor_attributes, outer_size, outer_stride):
        block_size, shape, quant_min, quant_max, zero_point_domain, dtype = tensor_attributes
        impl = _adopt_loaded_impl(tensor_data_dict["tensor_impl"],
                                  shape if outer_size is None else outer_size)
        return cls(
            impl,
            block_size,
            shape if outer_size is None else outer_size,
            quant_min,
            quant_max,
            zero_point_domain,
            dtype=dtype,
            strides=outer_stride,
        )

    def __setstate__(self, state):
        """Unpickling (torch.load): restore the fields, then let the layout adopt storage that
        another build wrote (a reference TensorCoreTiledLayout checkpoint holds the tile format;
        tensor_core_tiled_layout.convert_from_tensor_core_tiled)."""
        torch._utils._set_obj_state(self, state)
        self.tensor_impl = _adopt_loaded_impl(self.tensor_impl, self.shape)

    @classmethod
    def from_hp_to_intx(
        cls,
        input_float: torch.Tensor,
        mapping_type: MappingType,
        block_size: Tuple[int, ...],
        target_dtype: torch.dtype,
        quant_min: Optional[int] = None,
        quant_max: Optional[int] = None,
        eps: Optional[float] = None,
        scale_dtype: Optional[torch.dtype] = None,
        zero_point_dtype: Optional[torch.dtype] = None,
        preserve_zero: bool = True,
        zero_point_domain: ZeroPointDomain = ZeroPointDomain.INT,
        _layout: Layout = PlainLayout(),
        use_hqq: bool = False,
    ):
        """Quantize a high-precision tensor into an integer AQT with ``_layout``."""
        if use_hqq:
            raise NotImplementedError("HQQ quantization is outside the MI355X hot-path scope")
        original_shape = input_float.shape
        input_float = _layout.pre_process(input_float)
        fused = _fused_weight_quant(
            input_float, mapping_type, block_size, target_dtype, quant_min, quant_max, eps,
            scale_dtype, zero_point_dtype, preserve_zero, zero_point_domain, _layout,
        )
        if fused is not None:
            return cls(
                fused,
                block_size,
                original_shape,
                quant_min,
                quant_max,
                zero_point_domain,
                dtype=input_float.dtype,
            )
        if zero_point_domain == ZeroPointDomain.FLOAT and not preserve_zero:
            scale, zero_point = _choose_qparams_affine_tinygemm(
                input_float, mapping_type, block_size, target_dtype, quant_min, quant_max, eps,
                scale_dtype, zero_point_dtype,
            )
        elif not preserve_zero:
            raise NotImplementedError(
                "preserve_zero=False with an integer zero point is outside the hot-path scope"
            )
        else:
            scale, zero_point = choose_qparams_affine(
                input_float, mapping_type, block_size, target_dtype, quant_min, quant_max, eps,
                scale_dtype, zero_point_dtype,
            )
        if zero_point_domain == ZeroPointDomain.NONE:
            zero_point = None
            data = _quantize_affine_no_zero_point(
                input_float, block_size, scale, zero_point, target_dtype, quant_min, quant_max
            )
        elif zero_point_domain == ZeroPointDomain.FLOAT:
            data = _quantize_affine_tinygemm(
                input_float, block_size, scale, zero_point, target_dtype, quant_min, quant_max
            )
        else:
            data = quantize_affine(
                input_float, block_size, scale, zero_point, target_dtype, quant_min, quant_max
            )
        data, scale, zero_point = _layout.post_process(data, scale, zero_point, block_size)
        tensor_impl = cls.get_tensor_impl_constructor(type(_layout))(
            data, scale, zero_point, _layout
        )
        return cls(
            tensor_impl,
            block_size,
            original_shape,
            quant_min,
            quant_max,
            zero_point_domain,
            dtype=input_float.dtype,
        )

    @classmethod
    def from_hp_to_intx_static(
        cls,
        input_float: torch.Tensor,
        scale: torch.Tensor,
        zero_point: Optional[torch.Tensor],
        block_size: Tuple[int, ...],
        target_dtype: torch.dtype,
        quant_min: Optional[int] = None,
        quant_max: Optional[int] = None,
        zero_point_domain: ZeroPointDomain = ZeroPointDomain.INT,
        _layout: Layout = PlainLayout(),
    ):
        """Quantize with caller-supplied qparams."""
        if zero_point_domain is None:
            raise ValueError("please use ZeroPointDomain.NONE instead of None")
        if zero_point_domain is ZeroPointDomain.NONE and zero_point is not None:
            raise ValueError("zero_point should be None when zero_point_domain is NONE")
        original_shape = input_float.shape
        input_float, scale, zero_point = _layout.pre_process_static(
            input_float, scale, zero_point, block_size
        )
        if zero_point_domain == ZeroPointDomain.NONE:
            data = _quantize_affine_no_zero_point(
                input_float, block_size, scale, None, target_dtype, quant_min, quant_max
            )
        elif zero_point_domain == ZeroPointDomain.FLOAT:
            data = _quantize_affine_tinygemm(
                input_float, block_size, scale, zero_point, target_dtype, quant_min, quant_max
            )
        else:
            data = quantize_affine(
                input_float, block_size, scale, zero_point, target_dtype, quant_min, quant_max
            )
        data, scale, zero_point = _layout.post_process(data, scale, zero_point, block_size)
        tensor_impl = cls.get_tensor_impl_constructor(type(_layout))(
            data, scale, zero_point, _layout
        )
        return cls(
            tensor_impl,
            block_size,
            original_shape,
            quant_min,
            quant_max,
            zero_point_domain,
            dtype=input_float.dtype,
        )

    def to(self, *args, **kwargs):
        kwargs = self._get_to_kwargs(*args, **kwargs)
        device = kwargs.pop("device")
        return type(self)(
            self.tensor_impl.to(device),
            self.block_size,
            self.shape,
            self.quant_min,
            self.quant_max,
            self.zero_point_domain,
            **kwargs,
        )

    def _apply_fn_to_data(self, fn):
        return type(self)(
            fn(self.tensor_impl),
            self.block_size,
            self.shape,
            self.quant_min,
            self.quant_max,
            self.zero_point_domain,
            dtype=self.dtype,
            strides=self.stride(),
        )


register_layout = AffineQuantizedTensor.register_layout
get_tensor_impl_constructor = AffineQuantizedTensor.get_tensor_impl_constructor
to_affine_quantized_intx = AffineQuantizedTensor.from_hp_to_intx
to_affine_quantized_intx_static = AffineQuantizedTensor.from_hp_to_intx_static

torch.serialization.add_safe_globals([AffineQuantizedTensor])
