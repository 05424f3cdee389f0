"""``quantize_`` and the weight-only / dynamic-int8 workflow configs.

Reference: torchao/quantization/quant_api.py — ``quantize_`` (:482-546) walks the module tree
(:173-222) and swaps the weight of every module ``filter_fn`` selects (default ``_is_linear``,
:271-288) for a quantized tensor subclass, using the transform registered for the config type.
Configs on the MI355X hot path, with the reference defaults:

* ``Int4WeightOnlyConfig`` (:997-1158): uint4 asymmetric per-group, float zero point,
  ``TensorCoreTiledLayout(inner_k_tiles=8)`` -> gfx950 int4 kernels;
* ``Int8WeightOnlyConfig`` (:1200-1255): int8 symmetric per-channel -> int8 GEMV / MFMA;
* ``Int8DynamicActivationInt8WeightConfig`` (:1352-1449): int8 per-channel weight + per-token
  reduced-range int8 activation quantized on the fly -> HIP quant kernel + int8 MFMA GEMM.

Other workflows of the reference (float8, HQQ, fbgemm "version 2" tensors, marlin, gemlite,
intx, QAT, ...) are out of scope and raise.
"""

import logging
import types
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Optional, Tuple

import torch
import torch.nn as nn

import torchao
from torchao.core.config import AOBaseConfig
from torchao.dtypes.affine_quantized_tensor import (
    AffineQuantizedTensor,
    to_affine_quantized_intx,
)
from torchao.dtypes.uintx.plain_layout import PlainAQTTensorImpl
from torchao.dtypes.uintx.tensor_core_tiled_layout import TensorCoreTiledLayout
from torchao.dtypes.utils import Layout, PlainLayout
from torchao.quantization.linear_activation_quantized_tensor import (
    LinearActivationQuantizedTensor,
    to_linear_activation_quantized,
)
from torchao.quantization.quant_primitives import MappingType, ZeroPointDomain
from torchao.quantization.transform_module import (
    _QUANTIZE_CONFIG_HANDLER,
    register_quantize_module_handler,
)
from torchao.quantization.utils import _get_per_token_block_size

logger = logging.getLogger(__name__)

__all__ = [
    "quantize_",
    "Int4WeightOnlyConfig",
    "int4_weight_only",
    "Int8WeightOnlyConfig",
    "int8_weight_only",
    "Int8DynamicActivationInt8WeightConfig",
    "int8_dynamic_activation_int8_weight",
    "ModuleFqnToConfig",
    "LAYOUT_TO_ZERO_POINT_DOMAIN",
    "LAYOUT_TO_PRESERVE_ZEROS",
]

LAYOUT_TO_ZERO_POINT_DOMAIN = {TensorCoreTiledLayout: [ZeroPointDomain.FLOAT]}
LAYOUT_TO_PRESERVE_ZEROS = {TensorCoreTiledLayout: False}


# ---------------------------------------------------------------------------------------------
# module walking
# ---------------------------------------------------------------------------------------------
def _replace_with_custom_fn_if_matches_filter(
    model,
    replacement_fn,
    filter_fn,
    cur_fqn: str = "",
    device=None,
    extra_args: Optional[Tuple[Any, ...]] = (),
):
    """Depth-first: replace ``model`` itself if ``filter_fn(model, fqn)``, else recurse into
    its children (re-attaching replaced children). Moves modules to ``device`` first."""
    if filter_fn(model, cur_fqn[:-1]):
        if device is not None:
            model.to(device=device)
        return replacement_fn(model, *extra_args)
    for name, child in list(model.named_children()):
        new_child = _replace_with_custom_fn_if_matches_filter(
            child, replacement_fn, filter_fn, f"{cur_fqn}{name}.", device, extra_args
        )
        if new_child is not None and new_child is not child:
            setattr(model, name, new_child)
    if device is not None:
        model.to(device=device)
    return model


def _is_linear(mod, *args) -> bool:
    """An ``nn.Linear`` whose weight is not already quantized."""
    return (
        isinstance(mod, nn.Linear)
        and hasattr(mod, "weight")
        and not isinstance(mod.weight, (AffineQuantizedTensor, LinearActivationQuantizedTensor))
        and not isinstance(mod, nn.modules.linear.NonDynamicallyQuantizableLinear)
    )


def _quantization_type(weight: torch.Tensor) -> str:
    if isinstance(weight, AffineQuantizedTensor):
        return f"{type(weight).__name__}({weight._quantization_type()})"
    if isinstance(weight, LinearActivationQuantizedTensor):
        return (
            f"{type(weight).__name__}(activation={weight.input_quant_func}, "
            f"weight={_quantization_type(weight.original_weight_tensor)})"
        )
    if type(weight) is torch.Tensor or isinstance(weight, nn.Parameter):
        return f"Tensor: {type(weight)}"
    return f"not recognized: {type(weight)}"


def _linear_extra_repr(self):
    return (
        f"in_features={self.weight.shape[1]}, out_features={self.weight.shape[0]}, "
        f"weight={_quantization_type(self.weight)}"
    )


@dataclass
class ModuleFqnToConfig(AOBaseConfig):
    """Per-module configs by fully qualified name; ``"_default"`` applies to the rest."""

    module_fqn_to_config: Dict[str, Optional[AOBaseConfig]] = field(default_factory=dict)


def quantize_(
    model: nn.Module,
    config: AOBaseConfig,
    filter_fn: Optional[Callable[[nn.Module, str], bool]] = None,
    device: Optional[torch.types.Device] = None,
):
    """Quantize, in place, the weights of the modules of ``model`` that ``filter_fn`` selects.

    Example::

        m = nn.Sequential(nn.Linear(4096, 4096)).to(torch.bfloat16).cuda()
        quantize_(m, Int4WeightOnlyConfig(group_size=32))   # gfx950 int4 kernels
    """
    torch._C._log_api_usage_once("torchao.quantization.quantize_")
    filter_fn = _is_linear if filter_fn is None else filter_fn

    if isinstance(config, ModuleFqnToConfig):
        table = config.module_fqn_to_config

        def by_fqn(mod, fqn):
            cfg = table.get(fqn, table.get("_default", None))
            if cfg is None:
                return mod
            return _QUANTIZE_CONFIG_HANDLER[type(cfg)](mod, cfg)

        def walk(mod, prefix=""):
            for name, child in list(mod.named_children()):
                fqn = f"{prefix}{name}"
                if filter_fn(child, fqn):
                    if device is not None:
                        child.to(device=device)
                    setattr(mod, name, by_fqn(child, fqn))
                else:
                    walk(child, fqn + ".")

        walk(model)
        return

    if not isinstance(config, AOBaseConfig):
        raise AssertionError(
            "Passing a generic Callable to `quantize_` is not supported; pass a workflow config"
        )
    handler = _QUANTIZE_CONFIG_HANDLER[type(config)]
    _replace_with_custom_fn_if_matches_filter(
        model, handler, filter_fn, device=device, extra_args=(config,)
    )


# ---------------------------------------------------------------------------------------------
# int4 weight-only
# ---------------------------------------------------------------------------------------------
@dataclass
class Int4WeightOnlyConfig(AOBaseConfig):
    """uint4 asymmetric per-group weight-only quantization for the tinygemm-equivalent kernels.

    Args mirror the reference (quant_api.py:997-1040): ``group_size`` in {32, 64, 128, 256}
    (default 128), ``layout`` (default ``TensorCoreTiledLayout(inner_k_tiles=8)``),
    ``use_hqq`` (unsupported here), ``zero_point_domain`` (NONE = layout default, FLOAT),
    ``set_inductor_config``, ``preserve_zero`` (None = layout default, False), ``version``
    (1 = AffineQuantizedTensor; 2 = fbgemm tensors, unsupported).
    """

    group_size: int = 128
    layout: Optional[TensorCoreTiledLayout] = TensorCoreTiledLayout(inner_k_tiles=8)
    use_hqq: bool = False
    zero_point_domain: Optional[ZeroPointDomain] = ZeroPointDomain.NONE
    set_inductor_config: bool = True
    preserve_zero: Optional[bool] = None
    packing_format: str = "plain"
    version: int = 1

    def __post_init__(self):
        torch._C._log_api_usage_once("torchao.quantization.Int4WeightOnlyConfig")


int4_weight_only = Int4WeightOnlyConfig


def _int4_weight_only_quantize_tensor(weight: torch.Tensor, config: Int4WeightOnlyConfig):
    group_size = config.group_size
    layout = config.layout
    if weight.shape[-1] % group_size != 0:
        logger.info(
            f"Skipping quantizing weight with int4 weight only quantization because the shape "
            f"of weight {weight.shape} is not compatible with group_size {group_size}"
        )
        return weight
    if config.version != 1:
        raise NotImplementedError("Int4WeightOnlyConfig(version=2) (fbgemm tensors) is out of scope")
    if config.use_hqq:
        raise NotImplementedError("Int4WeightOnlyConfig(use_hqq=True) is out of scope")
    assert type(layout) in LAYOUT_TO_ZERO_POINT_DOMAIN, (
        f"Only support layout: {list(LAYOUT_TO_ZERO_POINT_DOMAIN)}"
    )
    zero_point_domain = config.zero_point_domain
    if zero_point_domain == ZeroPointDomain.NONE:
        zero_point_domain = LAYOUT_TO_ZERO_POINT_DOMAIN[type(layout)][0]
    assert zero_point_domain in LAYOUT_TO_ZERO_POINT_DOMAIN[type(layout)], (
        f"Layout only support {LAYOUT_TO_ZERO_POINT_DOMAIN[type(layout)]}"
    )
    preserve_zero = (
        config.preserve_zero
        if config.preserve_zero is not None
        else LAYOUT_TO_PRESERVE_ZEROS[type(layout)]
    )
    block_size = tuple([1] * (weight.ndim - 1) + [group_size])
    return to_affine_quantized_intx(
        weight,
        MappingType.ASYMMETRIC,
        block_size,
        torch.int32,
        0,
        15,
        1e-6,
        zero_point_dtype=torch.bfloat16,
        preserve_zero=preserve_zero,
        zero_point_domain=zero_point_domain,
        _layout=layout,
        use_hqq=config.use_hqq,
    )


def _swap_weight(module: nn.Module, new_weight: torch.Tensor) -> nn.Module:
    module.weight = nn.Parameter(new_weight, requires_grad=False)
    module.extra_repr = types.MethodType(_linear_extra_repr, module)
    return module


@register_quantize_module_handler(Int4WeightOnlyConfig)
def _int4_weight_only_transform(module: nn.Module, config: Int4WeightOnlyConfig) -> nn.Module:
    if config.set_inductor_config:
        torchao.quantization.utils.recommended_inductor_config_setter()
    assert hasattr(module, "weight"), "int4 weight-only quant requires a module with a weight"
    return _swap_weight(module, _int4_weight_only_quantize_tensor(module.weight, config))


# ---------------------------------------------------------------------------------------------
# int8 weight-only
# ---------------------------------------------------------------------------------------------
@dataclass
class Int8WeightOnlyConfig(AOBaseConfig):
    """int8 symmetric weight-only quantization, per channel (``group_size=None``) or per group."""

    group_size: Optional[int] = None
    set_inductor_config: bool = True

    def __post_init__(self):
        torch._C._log_api_usage_once("torchao.quantization.Int8WeightOnlyConfig")


int8_weight_only = Int8WeightOnlyConfig


def _int8_weight_only_quantize_tensor(weight: torch.Tensor, config: Int8WeightOnlyConfig):
    group_size = weight.shape[-1] if config.group_size is None else config.group_size
    block_size = tuple([1] * (weight.dim() - 1) + [group_size])
    return to_affine_quantized_intx(
        weight,
        MappingType.SYMMETRIC,
        block_size,
        torch.int8,
        eps=torch.finfo(torch.float32).eps,
        zero_point_dtype=torch.int64,
    )


@register_quantize_module_handler(Int8WeightOnlyConfig)
def _int8_weight_only_transform(module: nn.Module, config: Int8WeightOnlyConfig) -> nn.Module:
    if config.set_inductor_config:
        torchao.quantization.utils.recommended_inductor_config_setter()
    assert hasattr(module, "weight"), "int8 weight-only quant requires a module with a weight"
    return _swap_weight(module, _int8_weight_only_quantize_tensor(module.weight, config))


# ---------------------------------------------------------------------------------------------
# int8 dynamic activation x int8 weight
# ---------------------------------------------------------------------------------------------
def _int8_symm_per_token_reduced_range_quant(x: torch.Tensor) -> torch.Tensor:
    """Per-token symmetric int8 in [-127, 127], eps 1e-5 (reference quant_api.py:1258-1273).

    bf16 activations on the GPU run the fused HIP kernel (``torchao::int8_quantize_per_token``,
    bit-identical to the torch-op formulation); anything else uses the torch ops.
    """
    if x.is_cuda and x.dtype == torch.bfloat16 and x.shape[-1] % 16 == 0:
        q, s = torch.ops.torchao.int8_quantize_per_token(x)
        impl = PlainAQTTensorImpl(q, s, None, PlainLayout())
        return AffineQuantizedTensor(
            impl,
            tuple(_get_per_token_block_size(x)),
            x.shape,
            -127,
            127,
            ZeroPointDomain.INT,
            dtype=x.dtype,
        )
    return to_affine_quantized_intx(
        x,
        MappingType.SYMMETRIC,
        _get_per_token_block_size(x),
        torch.int8,
        eps=1e-5,
        quant_min=-127,
        quant_max=127,
        scale_dtype=torch.float32 if x.dtype == torch.float16 else None,
    )


def _int8_symm_per_token_reduced_range_quant_noop_decode(x: torch.Tensor) -> torch.Tensor:
    if x.dim() > 1 and x.shape[1] == 1:
        return x
    return _int8_symm_per_token_reduced_range_quant(x)


@dataclass
class Int8DynamicActivationInt8WeightConfig(AOBaseConfig):
    """int8 per-token dynamic activation x int8 per-channel weight (reference :1352-1372)."""

    layout: Optional[Layout] = PlainLayout()
    act_mapping_type: Optional[MappingType] = MappingType.SYMMETRIC
    weight_only_decode: bool = False
    set_inductor_config: bool = True

    def __post_init__(self):
        torch._C._log_api_usage_once("torchao.quantization.Int8DynamicActivationInt8WeightConfig")


int8_dynamic_activation_int8_weight = Int8DynamicActivationInt8WeightConfig


def _int8_dynamic_activation_int8_weight_quantize_tensor(weight, config):
    if weight.shape[-1] <= 16:
        logger.info(
            f"Skipping applying int8_dynamic_activation_int8_weight to weight of shape "
            f"{weight.shape} because `in_feature` is <= 16: {weight.shape[-1]}"
        )
        return weight
    if not isinstance(config.layout, PlainLayout):
        raise NotImplementedError("only PlainLayout is supported for int8 dynamic quantization")
    if config.act_mapping_type != MappingType.SYMMETRIC:
        raise NotImplementedError("asymmetric activation quantization is out of scope")
    input_quant_func = (
        _int8_symm_per_token_reduced_range_quant_noop_decode
        if config.weight_only_decode
        else _int8_symm_per_token_reduced_range_quant
    )
    block_size = tuple([1] * (weight.dim() - 1) + [weight.shape[-1]])
    new_weight = to_affine_quantized_intx(
        weight,
        MappingType.SYMMETRIC,
        block_size,
        torch.int8,
        eps=torch.finfo(torch.float32).eps,
        zero_point_dtype=torch.int64,
        _layout=config.layout,
        zero_point_domain=ZeroPointDomain.NONE,
    )
    return to_linear_activation_quantized(new_weight, input_quant_func)


@register_quantize_module_handler(Int8DynamicActivationInt8WeightConfig)
def _int8_dynamic_activation_int8_weight_transform(
    module: nn.Module, config: Int8DynamicActivationInt8WeightConfig
) -> nn.Module:
    if config.set_inductor_config:
        torchao.quantization.utils.recommended_inductor_config_setter()
    assert hasattr(module, "weight"), "int8 dynamic quant requires a module with a weight"
    return _swap_weight(
        module, _int8_dynamic_activation_int8_weight_quantize_tensor(module.weight, config)
    )
