"""Quantization helpers on the hot path (reference torchao/quantization/utils.py).

* ``pack_tinygemm_scales_and_zeros`` / ``unpack_tinygemm_scales_and_zeros`` (:395-414): the
  reference tile-format packing ``[K/g, N, 2]``, kept for the tile-format compat ops;
* ``pack_scales_and_zeros_gfx950`` / ``unpack_scales_and_zeros_gfx950``: the ``[N, K/g, 2]``
  interleaving the gfx950 row-stream kernels read (one dword per (row, group));
* ``compute_error`` (SQNR in dB, :53-56), ``_get_per_token_block_size`` (:141-146),
  ``recommended_inductor_config_setter`` (:665-680).
"""

from typing import List

import torch

__all__ = [
    "compute_error",
    "pack_tinygemm_scales_and_zeros",
    "unpack_tinygemm_scales_and_zeros",
    "pack_scales_and_zeros_gfx950",
    "unpack_scales_and_zeros_gfx950",
    "recommended_inductor_config_setter",
]


def compute_error(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """SQNR of ``y`` against reference ``x`` in dB: 20 log10(||x|| / ||x - y||)."""
    return 20 * torch.log10(torch.linalg.norm(x) / torch.linalg.norm(x - y))


def _check_same(t: torch.Tensor, name: str, dtype, size=None):
    if t.dtype != dtype:
        raise ValueError(f"Expected Tensor argument {name} to have dtype {dtype}, got {t.dtype}")
    if size is not None and t.size() != size:
        raise ValueError(f"Expected Tensor argument {name} to have size {size}, got {t.size()}")


def pack_tinygemm_scales_and_zeros(scales, zeros, dtype=torch.bfloat16):
    """(s, z) each [N, K/g] -> [K/g, N, 2] (the reference tinygemm / tile-format packing)."""
    _check_same(scales, "scales", dtype, zeros.size())
    _check_same(zeros, "zeros", dtype)
    return torch.stack([scales, zeros], dim=-1).transpose(-3, -2).contiguous()


def unpack_tinygemm_scales_and_zeros(scales_and_zeros):
    assert scales_and_zeros.shape[-1] == 2
    return torch.split(scales_and_zeros.transpose(-3, -2), 1, -1)


def pack_scales_and_zeros_gfx950(scales, zeros, dtype=torch.bfloat16):
    """(s, z) each [N, K/g] -> [N, K/g, 2]: one (scale, zero) dword per (row, group), read
    by the same lane that reads that group's nibbles."""
    _check_same(scales, "scales", dtype, zeros.size())
    _check_same(zeros, "zeros", dtype)
    return torch.stack([scales, zeros], dim=-1).contiguous()


def unpack_scales_and_zeros_gfx950(scales_and_zeros):
    assert scales_and_zeros.shape[-1] == 2
    return scales_and_zeros[..., 0], scales_and_zeros[..., 1]


def _get_per_token_block_size(x: torch.Tensor) -> List[int]:
    return [1] * (x.dim() - 1) + [x.shape[-1]]


def recommended_inductor_config_setter():
    """Inductor knobs the reference sets as a side effect of quantization (kept for parity)."""
    torch._inductor.config.coordinate_descent_tuning = True
    torch._inductor.config.coordinate_descent_check_all_directions = True
    torch._inductor.config.force_fuse_int_mm_with_mul = True
    torch._inductor.config.fx_graph_cache = True
    torch._inductor.config.triton.unique_kernel_names = True
    torch.set_float32_matmul_precision("high")
