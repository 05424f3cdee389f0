"""Layout plug-in base classes (reference torchao/dtypes/utils.py).

A ``Layout`` describes how an ``AffineQuantizedTensor`` stores its quantized data and which
kernels consume it; an ``AQTTensorImpl`` subclass registered for that layout
(``@AffineQuantizedTensor.register_layout(LayoutCls)``) implements ``from_plain`` (pack) and
``get_plain`` (unpack) plus the aten ops the tensor needs.
"""

from dataclasses import dataclass
from typing import Optional, Tuple, Union

import torch

from torchao.utils import TorchAOBaseTensor

__all__ = ["Layout", "PlainLayout", "AQTTensorImpl", "is_device", "get_out_shape"]


@dataclass(frozen=True)
class Layout:
    """Base layout: hooks to pad/reshape before quantization and after it."""

    def pre_process(self, input: torch.Tensor) -> torch.Tensor:
        return input

    def post_process(
        self,
        input: torch.Tensor,
        scale: torch.Tensor,
        zero_point: torch.Tensor,
        block_size: Tuple[int, ...],
    ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        return input, scale, zero_point

    def pre_process_static(
        self,
        input: torch.Tensor,
        scale: torch.Tensor,
        zero_point: torch.Tensor,
        block_size: Tuple[int, ...],
    ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        return self.pre_process(input), scale, zero_point

    def __repr__(self):
        return f"{type(self).__name__}({self.extra_repr()})"

    def extra_repr(self) -> str:
        return ""


@dataclass(frozen=True)
class PlainLayout(Layout):
    """Quantized data kept as plain (int_data, scale, zero_point) tensors."""


def is_device(target_device_str: str, device: Union[str, torch.device]) -> bool:
    return torch.device(device).type == target_device_str


def get_out_shape(input_shape, weight_shape):
    return (*input_shape[:-1], weight_shape[0])


class AQTTensorImpl(TorchAOBaseTensor):
    """Storage of an ``AffineQuantizedTensor`` for one layout."""

    def get_plain(self) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
        raise NotImplementedError

    def get_layout(self) -> Layout:
        return self._layout

    @classmethod
    def from_plain(cls, data, scale, zero_point, _layout: Layout):
        raise NotImplementedError

    def __repr__(self):
        data, scale, zero_point = self.get_plain()
        return (
            f"{type(self).__name__}(data={data}... , scale={scale}... , "
            f"zero_point={zero_point}... , _layout={self.get_layout()})"
        )
