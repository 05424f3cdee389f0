"""Tensor-subclass plumbing and small helpers shared by the quantized-linear path.

Mirrors the parts of the reference ``torchao/utils.py`` the hot path depends on:
``TorchAOBaseTensor`` with per-class op tables (utils.py:693-888), ``_implements``
(:435-470), the ``__torch_function__`` / ``__torch_dispatch__`` dispatchers (:576-615),
layout registration (:618-669), ``find_multiple`` (:177-181), ``fill_defaults``,
``benchmark_model`` (:69-122), ``get_model_size_in_bytes`` (:247-274) and device probes
(``is_MI350``, :939-944).
"""

import functools
import time
from typing import Any, Callable, Dict, List, Optional

import torch

__all__ = [
    "TorchAOBaseTensor",
    "benchmark_model",
    "fill_defaults",
    "find_multiple",
    "get_model_size_in_bytes",
    "is_MI350",
    "is_ROCM",
]


def find_multiple(n: int, *args: int) -> int:
    """Smallest multiple of lcm(args) that is >= n."""
    k = 1
    for a in args:
        k = k * a // _gcd(k, a)
    return n if n % k == 0 else n + k - (n % k)


def _gcd(a: int, b: int) -> int:
    while b:
        a, b = b, a % b
    return a


def fill_defaults(args, n: int, defaults_tail: List[Any]):
    """Pad positional ``args`` to length ``n`` with the trailing defaults."""
    args = list(args)
    missing = n - len(args)
    if missing < 0 or missing > len(defaults_tail):
        raise RuntimeError(f"fill_defaults: cannot fill {len(args)} args up to {n}")
    return args + list(defaults_tail[len(defaults_tail) - missing :])


def is_ROCM() -> bool:
    return torch.version.hip is not None and torch.cuda.is_available()


def is_MI350() -> bool:
    """True on gfx950 (MI350/MI355X)."""
    if not is_ROCM():
        return False
    return "gfx950" in torch.cuda.get_device_properties(0).gcnArchName


def benchmark_model(model: Callable, num_runs: int, args=(), kwargs=None, device_type=None):
    """Average wall time (ms) of ``model(*args, **kwargs)`` over ``num_runs`` calls."""
    kwargs = kwargs or {}
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        torch.cuda.synchronize()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(num_runs):
            model(*args, **kwargs)
        end.record()
        torch.cuda.synchronize()
        return start.elapsed_time(end) / num_runs
    t0 = time.perf_counter()
    for _ in range(num_runs):
        model(*args, **kwargs)
    return (time.perf_counter() - t0) * 1e3 / num_runs


def get_model_size_in_bytes(model: torch.nn.Module, ignore_embeddings: bool = False) -> int:
    """Bytes of parameters + buffers, counting quantized subclasses by their inner tensors."""

    def tensor_bytes(t: torch.Tensor) -> int:
        inner = t.data if isinstance(t, torch.nn.Parameter) else t
        if type(inner) is not torch.Tensor and hasattr(inner, "__tensor_flatten__"):
            names, _ = inner.__tensor_flatten__()
            return sum(tensor_bytes(getattr(inner, n)) for n in names)
        return inner.numel() * inner.element_size()

    total = 0
    for mod in model.modules():
        if ignore_embeddings and isinstance(mod, torch.nn.Embedding):
            continue
        for p in list(mod.parameters(recurse=False)) + list(mod.buffers(recurse=False)):
            total += tensor_bytes(p)
    return total


# --------------------------------------------------------------------------------------------
# op tables for tensor subclasses
# --------------------------------------------------------------------------------------------
def _implements(cls, aten_ops_or_torch_fns):
    """Decorator registering ``func(f, types, args, kwargs)`` for ops / torch functions."""
    table = cls.__dict__.get("_ATEN_OP_OR_TORCH_FN_TABLE_LOCAL")
    if table is None:
        table = {}
        setattr(cls, "_ATEN_OP_OR_TORCH_FN_TABLE_LOCAL", table)
    if not isinstance(aten_ops_or_torch_fns, (list, tuple)):
        aten_ops_or_torch_fns = [aten_ops_or_torch_fns]

    def decorator(fn):
        for op in aten_ops_or_torch_fns:
            table[op] = fn
        return fn

    return decorator


def _lookup(cls, func) -> Optional[Callable]:
    for klass in cls.__mro__:
        table = klass.__dict__.get("_ATEN_OP_OR_TORCH_FN_TABLE_LOCAL")
        if table is not None and func in table:
            return table[func]
    return None


def _dispatch__torch_function__(cls, func, types, args=(), kwargs=None):
    kwargs = kwargs or {}
    handler = _lookup(cls, func)
    if handler is not None:
        return handler(func, types, args, kwargs)
    with torch._C.DisableTorchFunctionSubclass():
        return func(*args, **kwargs)


def _dispatch__torch_dispatch__(cls, func, types, args, kwargs):
    handler = _lookup(cls, func)
    if handler is not None:
        return handler(func, types, args, kwargs or {})
    raise NotImplementedError(
        f"{cls.__name__} dispatch: attempting to run unimplemented operator/function: {func}"
    )


def _register_layout(tensor_class, layout_class):
    """``@Tensor.register_layout(LayoutCls)`` on a tensor-impl class: maps the layout to the
    impl's ``from_plain`` constructor and marks both safe for ``torch.load(weights_only=True)``."""

    def decorator(tensor_impl_class):
        table = tensor_class.__dict__.get("_LAYOUT_CONSTRUCTOR_TABLE")
        if table is None:
            table = {}
            setattr(tensor_class, "_LAYOUT_CONSTRUCTOR_TABLE", table)
        table[layout_class] = tensor_impl_class.from_plain
        torch.serialization.add_safe_globals([layout_class, tensor_impl_class])
        return tensor_impl_class

    return decorator


def _get_tensor_impl_constructor(tensor_class, layout_class) -> Callable:
    table = tensor_class.__dict__.get("_LAYOUT_CONSTRUCTOR_TABLE", {})
    if layout_class not in table:
        raise ValueError(f"layout_name: {layout_class} is not supported yet for {tensor_class}")
    return table[layout_class]


def _get_to_kwargs(self, *args, **kwargs):
    kwargs.pop("layout", None)
    args = tuple(a for a in args if not isinstance(a, torch.layout))
    device, dtype, _, _ = torch._C._nn._parse_to(*args, **kwargs)
    return {
        "device": self.device if device is None else device,
        "dtype": self.dtype if dtype is None else dtype,
    }


class TorchAOBaseTensor(torch.Tensor):
    """Base for torchao tensor subclasses: per-class op tables (inherited along the MRO),
    ``implements``, ``register_layout`` / ``get_tensor_impl_constructor``, ``_get_to_kwargs``."""

    implements = classmethod(_implements)
    __torch_dispatch__ = classmethod(_dispatch__torch_dispatch__)
    __torch_function__ = classmethod(_dispatch__torch_function__)
    register_layout = classmethod(_register_layout)
    get_tensor_impl_constructor = classmethod(_get_tensor_impl_constructor)
    _get_to_kwargs = _get_to_kwargs

    def get_layout(self):
        return getattr(self, "_layout", None)


@functools.lru_cache(maxsize=None)
def _device_arch(index: int = 0) -> str:
    return torch.cuda.get_device_properties(index).gcnArchName


def check_cpu_version(device) -> bool:
    return torch.device(device).type == "cpu"

