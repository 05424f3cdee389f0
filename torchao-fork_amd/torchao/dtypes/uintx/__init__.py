from .plain_layout import PlainAQTTensorImpl
from .tensor_core_tiled_layout import TensorCoreTiledAQTTensorImpl, TensorCoreTiledLayout

__all__ = ["PlainAQTTensorImpl", "TensorCoreTiledAQTTensorImpl", "TensorCoreTiledLayout"]
