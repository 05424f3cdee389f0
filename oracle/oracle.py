"""CPU oracle for the MI355X weight-only quantized linear path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / the timed CPU baseline. The product path (torchao-fork_amd/torchao) never
imports it: a GPU op whose native library is missing raises instead of falling back here.

What it restates (CPU, torch ops in bf16 with the reference's op order; numpy for byte work):

  int4 tinygemm (Int4WeightOnlyConfig):
    int4_qparams      <- _choose_qparams_affine_tinygemm   quant_primitives.py:1238-1307
    int4_quantize     <- _quantize_affine_tinygemm_no_dtype_cast   quant_primitives.py:544-573
    int4_dequantize   <- _dequantize_affine_tinygemm_no_dtype_check quant_primitives.py:939-1031
    int4_linear       <- AQT.dequantize() -> F.linear fallback  affine_quantized_tensor_ops.py:283-296
    int4_tinygemm_cpu <- aten._weight_int4pack_mm_for_cpu (Int4CPULayout, int4_cpu_layout.py:281-316)
  int8 weight-only (Int8WeightOnlyConfig):
    int8_weight_qparams/int8_weight_quantize <- choose_qparams_affine SYMMETRIC / quantize_affine
                                                quant_primitives.py:1497-1577, 398-459
    int8wo_linear     <- _linear_fp_act_int8_weight_impl  plain_layout.py:250-266
  int8 dynamic activation (Int8DynamicActivationInt8WeightConfig):
    int8_act_quant    <- _int8_symm_per_token_reduced_range_quant  quant_api.py:1258-1273
    int8_dyn_weight   <- _int8_dynamic_activation_int8_weight_quantize_tensor quant_api.py:1376-1430
    int8_scaled_mm    <- _linear_int8_act_int8_weight_impl + int_scaled_matmul
                         plain_layout.py:281-315, kernel/intmm.py:108-143 (CPU and GPU epilogues)
  byte layouts (numpy):
    pack_row_stream / unpack_row_stream  <- the gfx950 layout of include/torchao_mi355x.h
    pack_tile / unpack_tile              <- reference tile format, semantics of
                                            csrc/cuda/tensor_core_tiled_layout/tensor_core_tiled_layout.cu:131-215
                                            (fmt "cuda"), or PyTorch-ROCm's aten producer (fmt "rocm")

Pinning: every float function here is checked bit-exactly (torch.equal) against fixtures the
reference itself produced in the build container (oracle/gen_golden.py -> tests/golden/*.npz).
The tile format cannot be produced by the reference on CPU (aten._convert_weight_to_int4pack
has no CPU kernel). pack_tile(fmt="cuda") is pinned to the reference unpack kernel's index math
(round trip + hand-checked vectors: pinned to source); pack_tile(fmt="rocm") is pinned to the
nibble map PyTorch-ROCm's aten._convert_weight_to_int4pack produced on the MI355X
(tests/golden/aten_tile_map_rocm.npz, every nibble of 15 (N, K, ikt) cases: pinned to a run),
and the GPU tests compare the HIP pack with that aten op directly.
"""

from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

BF16 = torch.bfloat16


# ---------------------------------------------------------------------------------------------
# int4 tinygemm
# ---------------------------------------------------------------------------------------------
def int4_qparams(w: torch.Tensor, group_size: int, eps: float = 1e-6) -> Tuple[torch.Tensor, torch.Tensor]:
    """(scale, zero) [N, K/g] in w.dtype: s = clamp((max-min)/15, eps); z = min + 8 s."""
    N, K = w.shape
    wg = w.reshape(N, K // group_size, group_size)
    mn = torch.amin(wg, dim=-1)
    mx = torch.amax(wg, dim=-1)
    s = torch.clamp((mx - mn) / float(15 - 0), min=eps)
    z = mn + s * 8.0
    return s.to(w.dtype), z.to(w.dtype)


def int4_quantize(w: torch.Tensor, s: torch.Tensor, z: torch.Tensor, group_size: int) -> torch.Tensor:
    """q = clamp(round((w - (z - 8 s)) / s), 0, 15) as int32 [N, K]."""
    N, K = w.shape
    wg = w.reshape(N, K // group_size, group_size)
    lo = z.unsqueeze(-1) - s.unsqueeze(-1) * 8.0
    q = torch.clamp(torch.round((wg - lo) / s.unsqueeze(-1)), 0, 15)
    return q.reshape(N, K).to(torch.int32)


def int4_dequantize(q: torch.Tensor, s: torch.Tensor, z: torch.Tensor, group_size: int,
                    out_dtype=BF16) -> torch.Tensor:
    """w = bf16(bf16((q - 8)) * s) + z with two bf16 roundings (reference op order)."""
    N, K = q.shape
    d = (q.reshape(N, K // group_size, group_size) - 8.0).to(out_dtype)
    d *= s.unsqueeze(-1)
    d += z.unsqueeze(-1)
    return d.reshape(N, K)


def int4_linear(x: torch.Tensor, q, s, z, group_size: int, bias: Optional[torch.Tensor] = None):
    """The reference CPU "dequant path": dequantize -> F.linear in bf16."""
    return F.linear(x, int4_dequantize(q, s, z, group_size), bias)


def int4_linear_fp32(x, q, s, z, group_size, bias=None):
    """fp32 accumulation of the same dequantised weights (tolerance anchor)."""
    w = int4_dequantize(q, s, z, group_size).float()
    y = x.float() @ w.t()
    return y if bias is None else y + bias.float()


def int4_tinygemm_cpu_pack(q: torch.Tensor, s: torch.Tensor, z: torch.Tensor):
    """PyTorch's CPU int4 pack (what Int4CPULayout.from_plain does, int4_cpu_layout.py:103-126)."""
    packed = torch.ops.aten._convert_weight_to_int4pack_for_cpu(q.contiguous(), 1)
    sz = torch.stack([s, z], dim=-1).transpose(0, 1).contiguous()  # [K/g, N, 2]
    return packed, sz


def int4_tinygemm_cpu(x: torch.Tensor, packed, sz, group_size: int):
    """aten._weight_int4pack_mm_for_cpu (the reference's CPU int4 GEMM)."""
    return torch.ops.aten._weight_int4pack_mm_for_cpu(x.contiguous(), packed, group_size, sz)


# ---------------------------------------------------------------------------------------------
# int8 weight-only / dynamic activation
# ---------------------------------------------------------------------------------------------
def _sym_scale(t: torch.Tensor, qmin: int, qmax: int, eps: float) -> torch.Tensor:
    mn = torch.amin(t, dim=-1)
    mx = torch.amax(t, dim=-1)
    mn_neg = torch.min(mn, torch.zeros_like(mn))
    mx_pos = torch.max(mx, torch.zeros_like(mx))
    amax = torch.max(-mn_neg, mx_pos)
    return torch.clamp(amax / (float(qmax - qmin) / 2), min=eps)


def int8_weight_qparams(w: torch.Tensor) -> torch.Tensor:
    """Per-channel symmetric int8 scale [N] (dtype of w): clamp(amax / 127.5, f32 eps)."""
    return _sym_scale(w, -128, 127, torch.finfo(torch.float32).eps).to(w.dtype)


def int8_weight_quantize(w: torch.Tensor, s: torch.Tensor, qmin=-128, qmax=127) -> torch.Tensor:
    return torch.clamp(torch.round(w * (1.0 / s.unsqueeze(-1))), qmin, qmax).to(torch.int8)


def int8wo_linear(x, q, s, bias=None):
    """mm(x, q^T.to(x.dtype)) * s (+ bias): three bf16 roundings."""
    x2 = x.reshape(-1, x.shape[-1])
    m = torch.mm(x2, q.t().to(x.dtype))
    y = m * s.to(m.dtype)
    y = y.reshape(*x.shape[:-1], y.shape[-1])
    if bias is not None:
        y = y + bias.to(m.dtype)
    return y


def int8_act_quant(x: torch.Tensor):
    """Per-token reduced-range int8: s = clamp(amax/127, 1e-5) [M, 1]; q in [-127, 127]."""
    s = _sym_scale(x, -127, 127, 1e-5).to(x.dtype)
    q = torch.clamp(torch.round(x * (1.0 / s.unsqueeze(-1))), -127, 127).to(torch.int8)
    return q, s.unsqueeze(-1)


def int8_dyn_weight(w: torch.Tensor):
    s = int8_weight_qparams(w)
    return int8_weight_quantize(w, s), s


def int8_scaled_mm(xq, xs, wq, ws, bias=None, epilogue: str = "cpu"):
    """y = ((xq @ wq^T) * xs) * ws (+ bias) in bf16.

    epilogue="cpu": the reference CPU branch, int32 -> bf16 before the row scale
    (kernel/intmm.py:133-137) — the order the HIP kernel reproduces bit for bit;
    epilogue="fp32": float(int32) * row scale rounded once (a more accurate variant, used only
    as a tolerance anchor)."""
    x2 = xq.reshape(-1, xq.shape[-1])
    c = torch.mm(x2.to(torch.int64), wq.t().to(torch.int64))  # exact int accumulation
    xs2 = xs.reshape(-1, 1).to(BF16)
    if epilogue == "cpu":
        y = c.to(torch.int32).to(BF16) * xs2
    else:
        y = (c.to(torch.float32) * xs2.to(torch.float32)).to(BF16)
    y = y * ws.reshape(-1).to(BF16)
    y = y.reshape(*xq.shape[:-1], y.shape[-1])
    if bias is not None:
        y = y + bias
    return y


# ---------------------------------------------------------------------------------------------
# byte layouts (numpy)
# ---------------------------------------------------------------------------------------------
def pack_row_stream(q: np.ndarray) -> np.ndarray:
    """int [N, K] (0..15) -> uint32 [N, K/8]; bits 4i = q[8d+2i], bits 16+4i = q[8d+2i+1]."""
    q = np.asarray(q, dtype=np.uint32)
    N, K = q.shape
    g = q.reshape(N, K // 8, 4, 2)
    out = np.zeros((N, K // 8), dtype=np.uint32)
    for i in range(4):
        out |= g[:, :, i, 0] << np.uint32(4 * i)
        out |= g[:, :, i, 1] << np.uint32(16 + 4 * i)
    return out


def unpack_row_stream(p: np.ndarray) -> np.ndarray:
    p = np.asarray(p).view(np.uint32) if np.asarray(p).dtype != np.uint32 else np.asarray(p)
    N, KD = p.shape
    out = np.zeros((N, KD, 4, 2), dtype=np.int32)
    for i in range(4):
        out[:, :, i, 0] = (p >> np.uint32(4 * i)) & 0xF
        out[:, :, i, 1] = (p >> np.uint32(16 + 4 * i)) & 0xF
    return out.reshape(N, KD * 8)


def _tile_index(N: int, K: int, ikt: int, fmt: str = "cuda"):
    """For every element of the tile tensor [N/8][K/(ikt*16)][32][ikt/2]: (n, ks[4]).

    fmt "cuda": tensor_core_tiled_layout.cu:131-215 (the reference's own kernels).
    fmt "rocm": PyTorch-ROCm's aten._convert_weight_to_int4pack on gfx950, recovered on the box
    (experiments/probe_aten_tile_map.py) and pinned by tests/golden/aten_tile_map_rocm.npz: the
    same bytes seen flat as [N/16][K/(ikt*16)][64][ikt/2]; lane l: n = 16 nb + l % 16,
    b = kb*ikt*16 + 32 j + 4 (l // 16), ks = {b, b+2, b+16, b+18}."""
    KT = K // (ikt * 16)
    if fmt == "rocm":
        nb, kb, l, j = np.meshgrid(np.arange(N // 16), np.arange(KT), np.arange(64),
                                   np.arange(ikt // 2), indexing="ij")
        n = nb * 16 + l % 16
        b = kb * ikt * 16 + 32 * j + 4 * (l // 16)
        ks = np.stack([b, b + 2, b + 16, b + 18], -1)
        shape = (N // 8, KT, 32, ikt // 2)
        return n.reshape(shape), ks.reshape(*shape, 4)
    nt, kt, t, j = np.meshgrid(
        np.arange(N // 8), np.arange(KT), np.arange(32), np.arange(ikt // 2), indexing="ij"
    )
    n = nt * 8 + t // 4
    kb0 = (kt * ikt + 2 * j) * 16
    t4 = t % 4
    ks = np.stack([kb0 + 2 * t4, kb0 + 2 * t4 + 8, kb0 + 16 + 2 * t4, kb0 + 16 + 2 * t4 + 8], -1)
    return n, ks


def pack_tile(q: np.ndarray, ikt: int, fmt: str = "cuda") -> np.ndarray:
    """int [N, K] -> int32 tile tensor; bits 4i = q[n][ks_i], bits 16+4i = q[n][ks_i + 1]."""
    q = np.asarray(q, dtype=np.uint32)
    N, K = q.shape
    n, ks = _tile_index(N, K, ikt, fmt)
    out = np.zeros(n.shape, dtype=np.uint32)
    for i in range(4):
        out |= q[n, ks[..., i]] << np.uint32(4 * i)
        out |= q[n, ks[..., i] + 1] << np.uint32(16 + 4 * i)
    return out.view(np.int32)


def unpack_tile(p: np.ndarray, ikt: int, fmt: str = "cuda") -> np.ndarray:
    p = np.asarray(p).view(np.uint32)
    N = p.shape[0] * 8
    K = p.shape[1] * ikt * 16
    n, ks = _tile_index(N, K, ikt, fmt)
    out = np.zeros((N, K), dtype=np.int32)
    for i in range(4):
        out[n, ks[..., i]] = (p >> np.uint32(4 * i)) & 0xF
        out[n, ks[..., i] + 1] = (p >> np.uint32(16 + 4 * i)) & 0xF
    return out


def dequant_tile_fma(q: torch.Tensor, sz_tiny: torch.Tensor, group_size: int) -> torch.Tensor:
    """Tile-format dequant semantics (one rounding): bf16(fma(q - 8, s, z)), sz [K/g, N, 2]."""
    N, K = q.shape
    s = sz_tiny[..., 0].t().float().repeat_interleave(group_size, dim=1)
    z = sz_tiny[..., 1].t().float().repeat_interleave(group_size, dim=1)
    w = (q.double() - 8.0) * s.double() + z.double()  # exact product; one rounding to f32
    return w.float().to(BF16)


# ---------------------------------------------------------------------------------------------
# inputs
# ---------------------------------------------------------------------------------------------
def make_linear_weight(N: int, K: int, seed: int = 0, dtype=BF16) -> torch.Tensor:
    """nn.Linear default init U(-1/sqrt(K), 1/sqrt(K)), deterministic on CPU."""
    g = torch.Generator().manual_seed(seed)
    bound = 1.0 / (K ** 0.5)
    return (torch.rand(N, K, generator=g, dtype=torch.float32) * 2 - 1).mul_(bound).to(dtype)


def make_activation(M: int, K: int, seed: int = 1, dtype=BF16) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randn(M, K, generator=g, dtype=torch.float32).to(dtype)


def rel_l2(y: torch.Tensor, ref: torch.Tensor) -> float:
    y, ref = y.double(), ref.double()
    return float(torch.linalg.norm(y - ref) / torch.linalg.norm(ref).clamp_min(1e-30))
