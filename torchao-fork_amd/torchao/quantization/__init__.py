"""Quantization workflows on the MI355X weight-only linear path."""

from torchao.quantization.fuse import fuse_gate_up_
from torchao.quantization.linear_activation_quantized_tensor import (
    LinearActivationQuantizedTensor,
    to_linear_activation_quantized,
)
from torchao.quantization.quant_api import (
    Int4WeightOnlyConfig,
    Int8DynamicActivationInt8WeightConfig,
    Int8WeightOnlyConfig,
    ModuleFqnToConfig,
    int4_weight_only,
    int8_dynamic_activation_int8_weight,
    int8_weight_only,
    quantize_,
)
from torchao.quantization.quant_primitives import (
    MappingType,
    ZeroPointDomain,
    choose_qparams_affine,
    dequantize_affine,
    quantize_affine,
)
from torchao.quantization.transform_module import register_quantize_module_handler
from torchao.quantization.utils import compute_error

__all__ = [
    "quantize_",
    "fuse_gate_up_",
    "Int4WeightOnlyConfig",
    "Int8WeightOnlyConfig",
    "Int8DynamicActivationInt8WeightConfig",
    "ModuleFqnToConfig",
    "int4_weight_only",
    "int8_weight_only",
    "int8_dynamic_activation_int8_weight",
    "LinearActivationQuantizedTensor",
    "to_linear_activation_quantized",
    "MappingType",
    "ZeroPointDomain",
    "choose_qparams_affine",
    "quantize_affine",
    "dequantize_affine",
    "register_quantize_module_handler",
    "compute_error",
]
