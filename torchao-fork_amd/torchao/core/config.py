"""Workflow configuration base class (reference torchao/core/config.py:27-67).

A config is a dataclass; ``quantize_`` looks up the module transform registered for its type
(``torchao.quantization.transform_module``). ``version`` is an instance field so configs of
different versions can coexist in a checkpoint. JSON (de)serialization of configs is out of scope
(SURVEY §2 row 7).
"""

import abc

_DEFAULT_VERSION = 1


class AOBaseConfig(abc.ABC):
    """Base of every workflow config accepted by ``torchao.quantization.quantize_``."""

    version: int = _DEFAULT_VERSION
