"""Quantization helpers on the hot path (reference torchao/quantization/utils.py).

* ``pack_tinygemm_scales_and_zeros`` / ``unpack_tinygemm_scales_and_zeros`` (:395-414): the
  reference tile-format packing ``[K/g, N, 2]``, kept for the tile-format compat ops;
* ``pack_scales_and_zeros_gfx950`` / ``unpack_scales_and_zeros_gfx950``: the ``[N, K/g, 2]``
  interleaving the gfx950 row-stream kernels read (one dword per (row, group));
* ``get_groupwise_affine_qparams`` / ``groupwise_affine_quantize_tensor_from_qparams`` /
  ``groupwise_affine_dequantize_tensor_from_qparams`` (:325-513): the group-wise int4 helpers the
  reference's tile-layout tests are written with (float zero-point domain = tinygemm; nibbles
  packed ``q[2i] << 4 | q[2i+1]`` into uint8 on a GPU device, int32 kept on the host);
* ``compute_error`` (SQNR in dB, :53-56), ``_get_per_token_block_size`` (:141-146),
  ``recommended_inductor_config_setter`` (:665-680).
"""

from typing import List

import torch

__all__ = [
    "compute_error",
    "get_groupwise_affine_qparams",
    "groupwise_affine_quantize_tensor_from_qparams",
    "groupwise_affine_dequantize_tensor_from_qparams",
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


def _int_mode(zero_point_domain):
    from torchao.quantization.quant_primitives import ZeroPointDomain
    if zero_point_domain not in (ZeroPointDomain.FLOAT, ZeroPointDomain.INT):
        raise ValueError(f"Unrecognized zero point domain: {zero_point_domain}")
    return zero_point_domain == ZeroPointDomain.INT


def get_groupwise_affine_qparams(w, n_bit=4, groupsize=128, dtype=torch.bfloat16,
                                 zero_point_domain=None, preserve_zero=False, eps=None):
    """Asymmetric per-(row, group) (scale, zero) of a 2-D weight, each [N, K/groupsize]
    (quantization/utils.py:326-391). The reference's three-way choice: float zero-point domain
    without zero preservation = the tinygemm scheme the int4 kernels consume; integer domain
    without it = _choose_qparams_affine_dont_preserve_zero; otherwise choose_qparams_affine
    (zero preserved)."""
    from torchao.quantization import quant_primitives as qp
    zero_point_domain = qp.ZeroPointDomain.FLOAT if zero_point_domain is None else zero_point_domain
    groupsize = min(groupsize, w.shape[-1])
    if not (groupsize > 1 and w.dim() == 2 and w.shape[-1] % groupsize == 0 and n_bit <= 8):
        raise ValueError(f"bad group-wise qparams request: {tuple(w.shape)}, g={groupsize}, "
                         f"n_bit={n_bit}")
    int_zero = _int_mode(zero_point_domain)
    zdt = torch.int32 if int_zero else dtype
    if not int_zero and not preserve_zero:
        choose = qp._choose_qparams_affine_tinygemm
    elif int_zero and not preserve_zero:
        choose = qp._choose_qparams_affine_dont_preserve_zero
    else:
        choose = qp.choose_qparams_affine
    scale, zero = choose(w, qp.MappingType.ASYMMETRIC, (1, groupsize), torch.int32, 0,
                         2 ** n_bit - 1, 1e-6 if eps is None else eps, scale_dtype=dtype,
                         zero_point_dtype=zdt)
    return scale.to(dtype).reshape(w.shape[0], -1), zero.to(zdt).reshape(w.shape[0], -1)


def groupwise_affine_quantize_tensor_from_qparams(w, scales, zeros, n_bit=4, groupsize=128,
                                                  zero_point_domain=None):
    """Quantize with given qparams. On a GPU device the int4 values come back two per byte
    (uint8 [N, K/2], high nibble first: the operand of aten._convert_weight_to_int4pack); on the
    host as int32 [N, K] (the CPU tinygemm operand)."""
    from torchao.quantization import quant_primitives as qp
    zero_point_domain = qp.ZeroPointDomain.FLOAT if zero_point_domain is None else zero_point_domain
    if groupsize > w.shape[-1] and scales.shape[-1] == 1:
        groupsize = w.shape[-1]
    if not (groupsize > 1 and w.dim() == 2 and w.shape[-1] % groupsize == 0):
        raise ValueError(f"bad group-wise quantize request: {tuple(w.shape)}, g={groupsize}")
    quant = qp.quantize_affine if _int_mode(zero_point_domain) else qp._quantize_affine_tinygemm
    q = quant(w, (1, groupsize), scales, zeros, torch.int32, 0, 2 ** n_bit - 1)
    if w.shape[-1] > 1 and w.device.type != "cpu":
        q = (q[:, ::2] << 4 | q[:, 1::2]).to(torch.uint8)
    return q


def groupwise_affine_dequantize_tensor_from_qparams(w_int4x8, scales, zeros, n_bit=4,
                                                    groupsize=128, zero_point_domain=None):
    """Inverse of the above (either storage form), in ``scales.dtype``; float domain: two
    roundings, (q - 2^(n-1)) * s then + z (quant_primitives._dequantize_affine_tinygemm)."""
    from torchao.quantization import quant_primitives as qp
    zero_point_domain = qp.ZeroPointDomain.FLOAT if zero_point_domain is None else zero_point_domain
    if w_int4x8.dim() != 2 or groupsize <= 1:
        raise ValueError("expected a 2-D quantized weight and groupsize > 1")
    q = w_int4x8
    if (q.dtype == torch.uint8 or q.shape[-1] > 1) and q.device.type != "cpu":
        b = q.to(torch.int32)
        q = torch.stack([b >> 4, b & 0x0F], dim=-1).reshape(b.shape[0], -1)
    if groupsize > q.shape[-1] and scales.shape[-1] == 1:
        groupsize = q.shape[-1]
    if q.shape[-1] % groupsize:
        raise ValueError(f"K ({q.shape[-1]}) is not a multiple of groupsize {groupsize}")
    deq = qp.dequantize_affine if _int_mode(zero_point_domain) else qp._dequantize_affine_tinygemm
    return deq(q, (1, groupsize), scales, zeros, torch.int32, 0, 2 ** n_bit - 1,
               output_dtype=scales.dtype)


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
