"""Registry from workflow-config type to module transform (reference transform_module.py:13-52)."""

import functools
from typing import Callable, Dict, Type

import torch

from torchao.core.config import AOBaseConfig

_QUANTIZE_CONFIG_HANDLER: Dict[
    Type[AOBaseConfig], Callable[[torch.nn.Module, AOBaseConfig], torch.nn.Module]
] = {}


def register_quantize_module_handler(config_type):
    """Decorator: ``@register_quantize_module_handler(MyConfig)`` on ``fn(module, config)``
    makes ``quantize_(model, MyConfig(...))`` call ``fn`` on every module the filter selects."""

    @functools.wraps(config_type)
    def decorator(func):
        _QUANTIZE_CONFIG_HANDLER[config_type] = func
        return func

    return decorator
