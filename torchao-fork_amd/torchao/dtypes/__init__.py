"""Quantized tensor subclasses and layouts of the MI355X weight-only linear path."""

from . import affine_quantized_tensor_ops  # noqa: F401  (registers the op overrides)
from .affine_quantized_tensor import (
    AffineQuantizedTensor,
    register_layout,
    to_affine_quantized_intx,
    to_affine_quantized_intx_static,
)
from .affine_quantized_tensor_ops import (
    QuantizedLinearNotImplementedError,
    deregister_aqt_quantized_linear_dispatch,
    register_aqt_quantized_linear_dispatch,
)
from .uintx import PlainAQTTensorImpl, TensorCoreTiledAQTTensorImpl, TensorCoreTiledLayout
from .utils import AQTTensorImpl, Layout, PlainLayout

__all__ = [
    "AffineQuantizedTensor",
    "AQTTensorImpl",
    "Layout",
    "PlainLayout",
    "PlainAQTTensorImpl",
    "TensorCoreTiledLayout",
    "TensorCoreTiledAQTTensorImpl",
    "QuantizedLinearNotImplementedError",
    "register_aqt_quantized_linear_dispatch",
    "deregister_aqt_quantized_linear_dispatch",
    "register_layout",
    "to_affine_quantized_intx",
    "to_affine_quantized_intx_static",
]
