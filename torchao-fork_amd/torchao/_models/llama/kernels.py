"""Python wrappers of the fused decode-step kernels (csrc/decode_ops.hip, C-ABI in
include/torchao_mi355x.h). Outputs are allocated with torch (graph-capture safe: inside a
capture they come from the graph's private pool); launches go on torch's current stream."""

import torch

from torchao import _lib

__all__ = ["rmsnorm", "rope_kv", "attn_decode", "silu_mul"]


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(t: torch.Tensor, dtype, name: str):
    if not t.is_cuda or t.dtype != dtype or not t.is_contiguous():
        raise RuntimeError(f"{name}: expected a contiguous CUDA {dtype} tensor, got "
                           f"{t.dtype} on {t.device} (contiguous={t.is_contiguous()})")


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    _check(x, torch.bfloat16, "rmsnorm x")
    _check(weight, torch.bfloat16, "rmsnorm weight")
    y = torch.empty_like(x)
    D = x.shape[-1]
    _lib.call("tao_rmsnorm_bf16", x.data_ptr(), weight.data_ptr(), y.data_ptr(), x.numel() // D,
              D, float(eps), _stream(x))
    return y


def rope_kv(qkv: torch.Tensor, freqs: torch.Tensor, pos: torch.Tensor, k_cache: torch.Tensor,
            v_cache: torch.Tensor, n_head: int) -> torch.Tensor:
    """qkv [B, S, (H + 2 Hkv) D] -> rotated q [B, H, S, D]; k, v written to the caches at pos."""
    _check(qkv, torch.bfloat16, "rope_kv qkv")
    _check(freqs, torch.float32, "rope_kv freqs")
    _check(pos, torch.int64, "rope_kv pos")
    B, S, _ = qkv.shape
    _, Hkv, T, D = k_cache.shape
    q = torch.empty(B, n_head, S, D, dtype=qkv.dtype, device=qkv.device)
    _lib.call("tao_rope_kv_bf16", qkv.data_ptr(), freqs.data_ptr(), pos.data_ptr(), q.data_ptr(),
              k_cache.data_ptr(), v_cache.data_ptr(), B, S, n_head, Hkv, D, T, _stream(qkv))
    return q


def attn_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                pos: torch.Tensor, scale: float) -> torch.Tensor:
    """q [B, H, 1, D] against keys 0..pos[0] -> [B, 1, H * D] bf16."""
    _check(q, torch.bfloat16, "attn_decode q")
    _check(pos, torch.int64, "attn_decode pos")
    B, H, S, D = q.shape
    assert S == 1, "attn_decode takes one query per (batch, head)"
    _, Hkv, T, _ = k_cache.shape
    nc = (T + 63) // 64
    part = torch.empty(B * Hkv * nc * (H // Hkv) * (D + 2), dtype=torch.float32, device=q.device)
    out = torch.empty(B, 1, H * D, dtype=q.dtype, device=q.device)
    _lib.call("tao_attn_decode_bf16", q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
              pos.data_ptr(), part.data_ptr(), out.data_ptr(), B, H, Hkv, D, T, float(scale),
              _stream(q))
    return out


def silu_mul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    _check(a, torch.bfloat16, "silu_mul a")
    _check(b, torch.bfloat16, "silu_mul b")
    y = torch.empty(a.shape, dtype=a.dtype, device=a.device)
    _lib.call("tao_silu_mul_bf16", a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(),
              _stream(a))
    return y
