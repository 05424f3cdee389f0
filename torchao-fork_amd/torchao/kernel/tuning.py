"""Scoped launch-shape overrides for the gfx950 kernels (sweeps and A/B measurements).

The C-ABI ``tao_tune_*`` hooks are thread-local (include/torchao_mi355x.h): an override only
re-routes launches issued from the thread that set it. ``tuning(...)`` sets overrides for a
``with`` block and restores every built-in choice (``tao_tune_reset``) on exit, so a sweep
cannot leave a production model re-routed.

    with tuning(gemm=(64, 2, 4), splitk_fenced=1):
        y = linear(x)
"""

import contextlib

from torchao import _lib

# keyword -> (entry point, number of int arguments)
_KNOBS = {
    "int4_gemv": ("tao_tune_int4_gemv", 4),
    "int4_lds": ("tao_tune_int4_lds", 1),
    "linear_crossover": ("tao_tune_linear_crossover", 1),
    "gemm": ("tao_tune_gemm", 3),
    "gemm_algo": ("tao_tune_gemm_algo", 1),
    "gemm_depth": ("tao_tune_gemm_depth", 1),
    "gemm_bn": ("tao_tune_gemm_bn", 1),
    "gemm_order": ("tao_tune_gemm_order", 1),
    "gemm_nw": ("tao_tune_gemm_nw", 1),
    "gemm_table": ("tao_tune_gemm_table", 1),
    "int4_mfma32": ("tao_tune_int4_mfma32", 1),
    "int4_xlds": ("tao_tune_int4_xlds", 1),
    "int4_norm": ("tao_tune_int4_norm", 1),
    "int8_gemv": ("tao_tune_int8_gemv", 3),
    "int8_quant": ("tao_tune_int8_quant", 1),
    "attn": ("tao_tune_attn", 1),
    "splitk_fenced": ("tao_tune_splitk_fenced", 1),
    "gemm_tile": ("tao_tune_gemm_tile", 2),
    "gemm_sf": ("tao_tune_gemm_sf", 7),
    "gemm_sf_seam": ("tao_tune_gemm_sf_seam", 1),
    "gemm_sf_loaders": ("tao_tune_gemm_sf_loaders", 1),
    "gemm_sf_xmap": ("tao_tune_gemm_sf_xmap", 1),
    "attn_prefill_nw": ("tao_tune_attn_prefill_nw", 1),
    "cnt_stride": ("tao_tune_cnt_stride", 1),
}


def apply(knob: str, *values: int) -> None:
    """Set one knob for the calling thread until ``reset()`` (measurement CLIs; prefer the scoped
    ``tuning`` form)."""
    if knob not in _KNOBS:
        raise ValueError(f"unknown tuning knob {knob!r}; known: {sorted(_KNOBS)}")
    name, nargs = _KNOBS[knob]
    if len(values) != nargs:
        raise ValueError(f"{knob} takes {nargs} value(s), got {len(values)}")
    _lib.call(name, *[int(a) for a in values])


def reset() -> None:
    """Restore every built-in launch choice for the calling thread."""
    _lib.call("tao_tune_reset")


@contextlib.contextmanager
def tuning(**knobs):
    """Apply ``knobs`` (names of ``_KNOBS``; a tuple for multi-argument hooks) inside the block,
    then reset to the built-in choices."""
    for k in knobs:
        if k not in _KNOBS:
            raise ValueError(f"unknown tuning knob {k!r}; known: {sorted(_KNOBS)}")
    try:
        for k, v in knobs.items():
            name, nargs = _KNOBS[k]
            args = tuple(v) if isinstance(v, (tuple, list)) else (v,)
            if len(args) != nargs:
                raise ValueError(f"{k} takes {nargs} value(s), got {len(args)}")
            _lib.call(name, *[int(a) for a in args])
        yield
    finally:
        reset()
