"""torchao (MI355X / gfx950 build) — weight-only quantized linear path.

API-compatible with the reference torchao 0.13.0 for ``quantize_`` with
``Int4WeightOnlyConfig`` / ``Int8WeightOnlyConfig`` / ``Int8DynamicActivationInt8WeightConfig``
and the ``AffineQuantizedTensor`` layout plug-in API. The compute runs in hand-written gfx950
HIP kernels behind a C-ABI library (``include/torchao_mi355x.h``), bound by ``torchao._lib`` and
exposed as ``torch.ops.torchao.*`` by ``torchao.ops`` (the reference loads ``_C*.so`` and imports
``ops`` the same way, torchao/__init__.py:26-32).
"""

import logging

import torch  # noqa: F401

__version__ = "0.13.0+mi355x"

logger = logging.getLogger(__name__)

from . import _lib  # noqa: E402
from . import ops  # noqa: E402,F401  (defines torch.ops.torchao.*; impls need the .so at call time)
from . import quantization  # noqa: E402  (first: dtypes imports quantization.quant_primitives)
from . import dtypes, kernel  # noqa: E402
from .quantization import quantize_  # noqa: E402

if not _lib.is_available():
    logger.debug("torchao MI355X native library not loaded: %s", _lib.load_error())

__all__ = ["dtypes", "kernel", "ops", "quantization", "quantize_"]
