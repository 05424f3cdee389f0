"""Python wrappers of the fused decode-step kernels (csrc/decode_ops.hip, C-ABI in
include/torchao_mi355x.h). Outputs are allocated with torch (graph-capture safe: inside a
capture they come from the graph's private pool); launches go on torch's current stream."""

from typing import Optional

import torch

from torchao import _lib

__all__ = ["rmsnorm", "rope_kv", "attn_decode", "silu_mul", "int4_linear_swiglu",
           "int4_linear_rope_kv", "int4_decode", "int8wo_decode", "int8dq_decode", "argmax",
           "argmax_advance", "check_decode_status"]


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


def add_rmsnorm(x: torch.Tensor, res: torch.Tensor, weight: torch.Tensor, eps: float):
    """(h, rmsnorm(h)) with h = x + res, in one launch (bit-identical to the two ops)."""
    _check(x, torch.bfloat16, "add_rmsnorm x")
    _check(res, torch.bfloat16, "add_rmsnorm res")
    _check(weight, torch.bfloat16, "add_rmsnorm weight")
    if res.shape != x.shape:
        raise RuntimeError(f"add_rmsnorm: shapes {tuple(x.shape)} and {tuple(res.shape)} differ")
    h, y = torch.empty_like(x), torch.empty_like(x)
    D = x.shape[-1]
    _lib.call("tao_add_rmsnorm_bf16", x.data_ptr(), res.data_ptr(), weight.data_ptr(),
              h.data_ptr(), y.data_ptr(), x.numel() // D, D, float(eps), _stream(x))
    return h, y


def add_rmsnorm_partials(x: torch.Tensor, part: torch.Tensor, weight: torch.Tensor, eps: float):
    """(h, rmsnorm(h)) with h = x + bf16(sum of the fp32 partial planes part [S, *x.shape]) in one
    launch (tao_add_rmsnorm_partials_bf16): bit-identical to add_rmsnorm(x, linear(...)) when
    part comes from int4_linear_partials of that linear."""
    _check(x, torch.bfloat16, "add_rmsnorm_partials x")
    _check(part, torch.float32, "add_rmsnorm_partials part")
    _check(weight, torch.bfloat16, "add_rmsnorm_partials weight")
    if tuple(part.shape[1:]) != tuple(x.shape):
        raise RuntimeError(f"add_rmsnorm_partials: part {tuple(part.shape)} does not hold planes "
                           f"of x {tuple(x.shape)}")
    h, y = torch.empty_like(x), torch.empty_like(x)
    D = x.shape[-1]
    _lib.call("tao_add_rmsnorm_partials_bf16", x.data_ptr(), part.data_ptr(), part.shape[0],
              weight.data_ptr(), h.data_ptr(), y.data_ptr(), x.numel() // D, D, float(eps),
              _stream(x))
    return h, y


def int4_linear_partials(x: torch.Tensor, packed: torch.Tensor, sz: torch.Tensor,
                         group_size: int) -> Optional[torch.Tensor]:
    """x @ W^T of an int4 linear as fp32 partial planes [S, *x.shape[:-1], N], one per K slice of
    the single-fetch GEMM, left for add_rmsnorm_partials to sum (no in-kernel split-K seam;
    tao_int4wo_linear_partials_f32), or None where the shape is not served that way."""
    import ctypes

    _check(x, torch.bfloat16, "int4_linear_partials x")
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M, K = x2.shape
    N = packed.shape[0]
    S = ctypes.c_int(0)
    _lib.call("tao_int4wo_linear_partial_slices", M, N, K, int(group_size),
              ctypes.cast(ctypes.pointer(S), ctypes.c_void_p))
    if S.value == 0:
        return None
    part = torch.empty(S.value, *x.shape[:-1], N, dtype=torch.float32, device=x.device)
    h = _lib.lib()
    rc = h.tao_int4wo_linear_partials_f32(x2.data_ptr(), packed.data_ptr(), sz.data_ptr(),
                                          part.data_ptr(), M, N, K, int(group_size), _stream(x))
    if rc == 2:  # TAO_ERR_UNSUPPORTED
        return None
    if rc != 0:
        raise RuntimeError(f"tao_int4wo_linear_partials_f32 failed (status {rc}): "
                           + h.tao_last_error().decode(errors="replace"))
    return part


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
    part = None
    if T > 1024:  # split-over-chunks path (shorter caches run one single-pass kernel)
        nc = (T + 63) // 64
        part = torch.empty(B * Hkv * nc * (H // Hkv) * (D + 2), dtype=torch.float32,
                           device=q.device)
    out = torch.empty(B, 1, H * D, dtype=q.dtype, device=q.device)
    _lib.call("tao_attn_decode_bf16", q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
              pos.data_ptr(), None if part is None else part.data_ptr(), out.data_ptr(), B, H,
              Hkv, D, T, float(scale), _stream(q))
    return out


# Decode attention split over key ranges (tao_attn_decode_split_bf16) with the merge folded into
# an int4 wo linear (tao_int4wo_attn_out_bf16): the splits per head (2 or 4; 0 = off, the one-pass
# kernel then the linear), taken for caches of ATTN_SPLIT_MIN_T..ATTN_SPLIT_MAX_T rows. Measured
# per layer (attention + wo, graph of 32 layers; profiles/r5a_attn_pair.jsonl): the split saves
# 1.1-4.4 us on the attention but the merge prologue costs wo ~1.5 us (every wo workgroup merges
# all heads' partials), so the pair pays only past ~600 keys: 328 keys one-pass 9.98 us vs
# 10.33 / 11.16 split 2 / 4; 512 keys 10.98 vs 10.83 / 11.38; 900 keys 14.29 vs 12.69 / 12.30;
# past 1024 rows against the two-launch chunk split: 1500 keys 23.3 vs 14.5, 3000 keys 35.1 vs
# 18.5 (split 4; profiles/r5b_attn_pair_long.jsonl). The route is chosen by the cache's
# capacity T (a graph is captured once per capacity, not per position), so it is taken only
# where every position gains: T > 1024, where the one-pass kernel's alternative is the two-launch
# chunk split; a 768-1024-row cache would run its early (short-history) steps slower on the pair.
ATTN_SPLITS = 4
ATTN_SPLIT_MIN_T = 1025
ATTN_SPLIT_MAX_T = 8192
PART_STRIDE = 132  # fp32 per (head, split) record: o[128], m, l, 2 pad


# Decode: RMSNorm -> wqkv -> RoPE + KV write and the decode attention in ONE launch
# (tao_int4wo_qkv_attn_bf16): the attention workgroups sit at the tail of the wqkv GEMV's grid,
# load their cache history while the GEMV streams, and start on the ticket of their q / kv heads
# instead of a stream-ordered launch. For int4 wqkv at batch 1, head_dim 128, caches of at most
# QKV_ATTN_MAX_T rows (each of the QKV_ATTN_SPLITS key ranges per head is walked by 4 waves).
# Off: measured SLOWER than the two launches (profiles/r5k_qkv_attn_time.jsonl, us per layer in a
# 32-layer graph, two launches vs one at 128 / 328 / 512 / 900 keys: 10.3 / 12.0 / 13.0 / 16.3 vs
# 13.0 / 13.5 / 13.6 / 16.3; e2e 721-729 vs 677-681 tok/s, r5k_ab_qkv_attn.jsonl): the in-launch
# chain of agent-scope hand-offs (q / k / v stores written through, ticket, poll, split partials,
# merge ticket) costs more than the launch boundary it removes.
DECODE_QKV_ATTN = False
QKV_ATTN_SPLITS = 4
QKV_ATTN_MAX_T = 2048


def qkv_attn_supported(N: int, K: int, n_head: int, n_kv_head: int, head_dim: int) -> bool:
    """Whether tao_int4wo_qkv_attn_bf16 serves this wqkv shape (its GEMV part runs the RMSNorm
    prologue's 4 waves x 2 rows launch shape)."""
    return bool(_lib.lib().tao_int4wo_qkv_attn_supported(N, K, n_head, n_kv_head, head_dim))


def int4_qkv_attn(x: torch.Tensor, packed: torch.Tensor, scale_and_zero: torch.Tensor,
                  group_size: int, norm_weight: torch.Tensor, eps: float, freqs: torch.Tensor,
                  pos: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, n_head: int,
                  scale: float, splits: int = 0) -> torch.Tensor:
    """One token: RMSNorm(x) -> int4 wqkv -> RoPE, k / v into the caches at pos[0], and the
    decode attention of the rotated q over keys 0..pos[0] -> [1, 1, n_head * D] bf16, in one
    launch (tao_int4wo_qkv_attn_bf16). Same results as int4_decode(..., "rope_kv") followed by
    attn_decode up to the attention's fp32 summation order."""
    _check(x, torch.bfloat16, "int4_qkv_attn x")
    _check(norm_weight, torch.bfloat16, "int4_qkv_attn norm_weight")
    _check(pos, torch.int64, "int4_qkv_attn pos")
    N, K = packed.shape[0], x.shape[-1]
    if x.numel() != K:
        raise RuntimeError(f"int4_qkv_attn takes one token, got x of shape {tuple(x.shape)}")
    B, Hkv, T, D = k_cache.shape
    if B != 1:
        raise RuntimeError("int4_qkv_attn: batch 1 caches only")
    q = torch.empty(1, n_head, 1, D, dtype=x.dtype, device=x.device)
    out = torch.empty(1, 1, n_head * D, dtype=x.dtype, device=x.device)
    _lib.call("tao_int4wo_qkv_attn_bf16", x.data_ptr(), packed.data_ptr(),
              scale_and_zero.data_ptr(), N, K, int(group_size), norm_weight.data_ptr(),
              float(eps), q.data_ptr(), out.data_ptr(), freqs.data_ptr(), pos.data_ptr(),
              k_cache.data_ptr(), v_cache.data_ptr(), n_head, Hkv, D, T, float(scale),
              int(splits or QKV_ATTN_SPLITS), _stream(x))
    return out


def int4_grouped_decode(x: torch.Tensor, packed: torch.Tensor, scale_and_zero: torch.Tensor,
                        group_size: int, expert_idx: torch.Tensor) -> torch.Tensor:
    """The A = expert_idx.numel() experts' int4 linears of one token in one launch
    (tao_int4wo_grouped_gemv_bf16): packed [E, N, K/8] int32, scale_and_zero [E, N, K/g, 2] bf16
    (a 3-D Int4WeightOnlyConfig weight's tensor_impl), x [K] / [1, K] (shared) or [A, K] (row a
    for expert a) bf16 -> y [A, N] bf16, row a bit-identical to expert expert_idx[a]'s linear."""
    _check(x, torch.bfloat16, "int4_grouped x")
    _check(expert_idx, torch.int64, "int4_grouped expert_idx")
    if packed.dim() != 3:
        raise RuntimeError(f"int4_grouped: packed must be [E, N, K/8], got {tuple(packed.shape)}")
    E, N, K8 = packed.shape
    K, A = K8 * 8, expert_idx.numel()
    rows = x.numel() // K
    if x.shape[-1] != K or rows not in (1, A):
        raise RuntimeError(f"int4_grouped: x {tuple(x.shape)} must be [K] or [A, K] with K = {K}")
    y = torch.empty(A, N, dtype=x.dtype, device=x.device)
    _lib.call("tao_int4wo_grouped_gemv_bf16", x.data_ptr(), rows, packed.data_ptr(),
              scale_and_zero.data_ptr(), expert_idx.data_ptr(), A, E, N, K, int(group_size),
              y.data_ptr(), _stream(x))
    return y


def int4_moe_ffn_decode(x: torch.Tensor, w1, w2, w3, expert_indices: torch.Tensor,
                        expert_weights: torch.Tensor) -> torch.Tensor:
    """The one-token branch of the reference's ConditionalFeedForwardAOQuantizable
    (_models/mixtral-moe/model.py:360-384) on 3-D int4 weights (AffineQuantizedTensor [E, I, D] /
    [E, D, I] / [E, I, D]): three grouped launches instead of 3 A per-expert linears, the same
    bf16 ops in between (silu(w1 x) * w3 x, then w2, then the expert-weighted sum)."""
    def parts(w):
        impl = w.tensor_impl
        return impl.packed_weight, impl.scale_and_zero, w.block_size[-1]

    idx = expert_indices.reshape(-1)
    y1 = torch.nn.functional.silu(int4_grouped_decode(x, *parts(w1), idx))
    y3 = int4_grouped_decode(x, *parts(w3), idx)
    y2 = int4_grouped_decode((y1 * y3).contiguous(), *parts(w2), idx)  # [A, D]
    return (y2 * expert_weights.view(-1, 1)).sum(dim=0).unsqueeze(-1)


def attn_decode_split(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                      pos: torch.Tensor, scale: float, splits: int) -> torch.Tensor:
    """q [B, H, 1, D] against keys 0..pos[0], the keys split `splits` ways per head ->
    unnormalised partials [B * H, splits, 132] fp32 (attn_merge or int4_attn_out finish it)."""
    _check(q, torch.bfloat16, "attn_decode q")
    _check(pos, torch.int64, "attn_decode pos")
    B, H, S, D = q.shape
    assert S == 1, "attn_decode takes one query per (batch, head)"
    _, Hkv, T, _ = k_cache.shape
    part = torch.empty(B * H, splits, PART_STRIDE, dtype=torch.float32, device=q.device)
    _lib.call("tao_attn_decode_split_bf16", q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
              pos.data_ptr(), part.data_ptr(), B, H, Hkv, D, T, float(scale), splits, _stream(q))
    return part


def attn_merge(part: torch.Tensor, B: int, H: int, D: int = 128) -> torch.Tensor:
    """The split partials merged -> [B, 1, H * D] bf16 (the one-pass kernel's output form)."""
    _check(part, torch.float32, "attn_merge partial")
    out = torch.empty(B, 1, H * D, dtype=torch.bfloat16, device=part.device)
    _lib.call("tao_attn_merge_bf16", part.data_ptr(), out.data_ptr(), B, H, D, part.shape[1],
              _stream(part))
    return out


def int4_attn_out(part: torch.Tensor, n_head: int, packed: torch.Tensor, sz: torch.Tensor,
                  group_size: int, residual=None) -> torch.Tensor:
    """wo at decode with the split merge as its x prologue: [1, 1, N] = bf16(bf16(W x) +
    residual), x = attn_merge(part) (batch 1)."""
    _check(part, torch.float32, "int4_attn_out partial")
    N, K = packed.shape[0], packed.shape[1] * 8
    y = torch.empty(1, 1, N, dtype=torch.bfloat16, device=part.device)
    if residual is not None:
        _check(residual, torch.bfloat16, "int4_attn_out residual")
        assert residual.numel() == N
    _lib.call("tao_int4wo_attn_out_bf16", part.data_ptr(), part.shape[1], n_head,
              packed.data_ptr(), sz.data_ptr(), N, K, group_size,
              None if residual is None else residual.data_ptr(), y.data_ptr(), _stream(part))
    return y


def attn_prefill(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                 pos: torch.Tensor, scale: float) -> torch.Tensor:
    """q [B, H, S, D] (query s at position pos[s]) against cache keys 0..pos[s] -> [B, S, H * D]
    bf16 (tao_attn_prefill_bf16): the causal-masked SDPA of a prompt over the caches."""
    _check(q, torch.bfloat16, "attn_prefill q")
    _check(pos, torch.int64, "attn_prefill pos")
    B, H, S, D = q.shape
    _, Hkv, T, _ = k_cache.shape
    if pos.numel() != S:
        raise RuntimeError(f"attn_prefill: {pos.numel()} positions for {S} queries")
    out = torch.empty(B, S, H * D, dtype=q.dtype, device=q.device)
    _lib.call("tao_attn_prefill_bf16", q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
              pos.data_ptr(), out.data_ptr(), B, H, Hkv, D, S, T, float(scale), _stream(q))
    return out


def int4_linear_swiglu(x: torch.Tensor, packed: torch.Tensor, sz: torch.Tensor,
                       group_size: int) -> Optional[torch.Tensor]:
    """silu_mul(x @ W^T) for an int4 w1||w3 weight with interleaved (gate, up) rows, the SiLU-mul
    folded into the GEMM's epilogue (tao_int4wo_linear_swiglu_bf16): [..., N / 2] bf16, or None
    where no fused kernel serves the shape (the caller runs the linear and silu_mul)."""
    _check(x, torch.bfloat16, "int4_linear_swiglu x")
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M, K = x2.shape
    N = packed.shape[0]
    y = torch.empty(*x.shape[:-1], N // 2, dtype=x.dtype, device=x.device)
    h = _lib.lib()
    rc = h.tao_int4wo_linear_swiglu_bf16(x2.data_ptr(), packed.data_ptr(), sz.data_ptr(),
                                         y.data_ptr(), M, N, K, int(group_size), _stream(x))
    if rc == 2:  # TAO_ERR_UNSUPPORTED
        return None
    if rc != 0:
        raise RuntimeError(f"tao_int4wo_linear_swiglu_bf16 failed (status {rc}): "
                           + h.tao_last_error().decode(errors="replace"))
    return y


def int4_linear_rope_kv(x: torch.Tensor, packed: torch.Tensor, sz: torch.Tensor,
                        group_size: int, freqs: torch.Tensor, pos: torch.Tensor,
                        k_cache: torch.Tensor, v_cache: torch.Tensor,
                        n_head: int) -> Optional[torch.Tensor]:
    """rope_kv(x @ Wqkv^T, ...) in one launch (tao_int4wo_linear_rope_kv_bf16): x [B, S, K] ->
    rotated q [B, H, S, D]; k, v written to the caches at pos. None where no fused kernel serves
    the shape (the caller runs the linear and rope_kv)."""
    _check(x, torch.bfloat16, "int4_linear_rope_kv x")
    _check(freqs, torch.float32, "int4_linear_rope_kv freqs")
    _check(pos, torch.int64, "int4_linear_rope_kv pos")
    B, S, K = x.shape
    _, Hkv, T, D = k_cache.shape
    if packed.shape[0] != (n_head + 2 * Hkv) * D:
        return None
    q = torch.empty(B, n_head, S, D, dtype=x.dtype, device=x.device)
    h = _lib.lib()
    rc = h.tao_int4wo_linear_rope_kv_bf16(x.data_ptr(), packed.data_ptr(), sz.data_ptr(), K,
                                          int(group_size), freqs.data_ptr(), pos.data_ptr(),
                                          q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), B,
                                          S, n_head, Hkv, D, T, _stream(x))
    if rc == 2:  # TAO_ERR_UNSUPPORTED
        return None
    if rc != 0:
        raise RuntimeError(f"tao_int4wo_linear_rope_kv_bf16 failed (status {rc}): "
                           + h.tao_last_error().decode(errors="replace"))
    return q


def silu_mul(a: torch.Tensor, b=None) -> torch.Tensor:
    """bf16(bf16(silu(a)) * b); with b None, ``a`` [..., 2n] holds interleaved (gate, up) pairs
    (an interleaved w13 output) and the result is [..., n]."""
    _check(a, torch.bfloat16, "silu_mul a")
    if b is None:
        y = torch.empty(*a.shape[:-1], a.shape[-1] // 2, dtype=a.dtype, device=a.device)
        _lib.call("tao_silu_mul_bf16", a.data_ptr(), None, y.data_ptr(), y.numel(), _stream(a))
        return y
    _check(b, torch.bfloat16, "silu_mul b")
    y = torch.empty(a.shape, dtype=a.dtype, device=a.device)
    _lib.call("tao_silu_mul_bf16", a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(),
              _stream(a))
    return y


_EPILOGUES = {"none": 0, "swiglu": 1, "rope_kv": 2}


# Prefill attention on tao_attn_prefill_bf16 (False: torch's masked SDPA over the caches).
PREFILL_ATTN = True
# Prefill residual adds fused with the following RMSNorm (tao_add_rmsnorm_bf16).
PREFILL_ADD_NORM = True
# Greedy prefill (Transformer.prefill_next) reads only the last position's hidden state: the last
# block runs wqkv + RoPE + KV write over every row (the caches need them) and everything after it
# for the last row only, on the one-token kernels (attention, wo + residual, RMSNorm + w1||w3 +
# SwiGLU, w2 + residual). Parity note: those kernels sum K in another order than the M = S GEMMs,
# so the first token is not bit-tied to the reference's model(idx)[:, -1].argmax; it agrees
# wherever the top-2 margin decides it (tests/test_llama_harness.py
# test_prefill_last_row_first_token_over_prompts_gpu); False (generate.py --prefill_last_row 0)
# restores the all-rows path.
PREFILL_LAST_ROW = True
# Prefill wo / w2 (int4, where the 16x16 single-fetch GEMM serves them): the K slices' fp32
# partial tiles are summed by the residual add + RMSNorm launch that follows instead of at an
# in-kernel split-K seam (int4_linear_partials + add_rmsnorm_partials; bit-identical).
PREFILL_PARTIALS = True

# Output heads (N >= HEAD_ROWS) normalise in their own RMSNorm launch unless HEAD_PROLOGUE.
HEAD_ROWS = 65536
HEAD_PROLOGUE = False


def prologue_pays(N: int, K: int) -> bool:
    """Whether the RMSNorm prologue inside the GEMV beats a separate RMSNorm launch: every
    workgroup of the GEMV re-normalises the row, so it pays while K or the grid is small.
    Measured (experiments/bench_decode.py; profiles/r1_bench_decode*.jsonl,
    r3_bench_decode_bpw.jsonl): Llama-3-8B wqkv and w1||w3 and 70B wqkv gain 1-6 µs; 70B
    w1||w3 (57344x8192) loses 3-9 µs; the vocabulary heads (128256 rows, 8016 workgroups) lose
    7.5 µs at K 4096 (round 3: fused 61.3 vs RMSNorm launch + GEMV 53.9 µs)."""
    if N >= HEAD_ROWS and not HEAD_PROLOGUE:
        return False
    return K <= 4096 or N < 16384


# Decode feed-forward (RMSNorm -> w1||w3 -> SwiGLU -> w2 -> + residual) in ONE persistent launch
# on the LDS-DMA engine (tao_int4wo_ffn_engine_bf16, csrc/decode_engine.hip) instead of the two
# fused GEMV launches, for int4 g32 at the shapes the engine serves (Llama-3-8B).
DECODE_FFN_ENGINE = False
_ENGINE_WS = {}


def ffn_engine_supported(dim: int, inter: int, group_size: int) -> bool:
    return bool(_lib.lib().tao_int4wo_ffn_engine_supported(dim, inter, group_size))


def ffn_engine_workspace(device: torch.device) -> torch.Tensor:
    """The engine's per-device workspace (epoch word, arrival counters, SwiGLU payload), created and initialised
    once, eagerly: its epoch advances on the device with every launch (graph replays included),
    so it must never be re-initialised by a captured op. Engine launches of one device must run
    on one stream at a time."""
    dev = torch.device(device)
    ws = _ENGINE_WS.get(dev)
    if ws is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("ffn engine: run once eagerly before graph capture (workspace)")
        nbytes = int(_lib.lib().tao_int4wo_ffn_engine_workspace_bytes(65536))
        ws = torch.zeros(nbytes // 4, dtype=torch.int32, device=dev)
        ws[0] = 1
        torch.cuda.synchronize(dev)
        _ENGINE_WS[dev] = ws
    return ws


def int4_ffn_engine(h: torch.Tensor, norm_weight: torch.Tensor, eps: float, w13: tuple,
                    w2: tuple) -> torch.Tensor:
    """One token through a Llama FFN with its residual, out = h + w2(swiglu(w13(rmsnorm(h)))),
    in one launch (tao_int4wo_ffn_engine_bf16). w13 / w2 = (packed, scale_and_zero, group_size)
    of the fused (w1_i, w3_i) int4 linear and of w2."""
    _check(h, torch.bfloat16, "ffn_engine h")
    _check(norm_weight, torch.bfloat16, "ffn_engine norm_weight")
    (p13, z13, g13), (p2, z2, g2) = w13, w2
    dim = h.shape[-1]
    inter = p13.shape[0] // 2
    if h.numel() != dim or g13 != g2 or p2.shape[0] != dim:
        raise RuntimeError("ffn_engine: one token, matching group sizes and shapes")
    ws = ffn_engine_workspace(h.device)
    out = torch.empty_like(h)
    base = ws.data_ptr()
    _lib.call("tao_int4wo_ffn_engine_bf16", h.data_ptr(), norm_weight.data_ptr(), float(eps),
              p13.data_ptr(), z13.data_ptr(), p2.data_ptr(), z2.data_ptr(), out.data_ptr(), dim,
              inter, int(g13), base, base + 4096, _stream(h))
    return out


def int4_decode(x: torch.Tensor, packed: torch.Tensor, scale_and_zero: torch.Tensor,
                group_size: int, norm_weight=None, eps: float = 0.0, epilogue: str = "none",
                rope=None) -> torch.Tensor:
    """One token through an int4 linear with its neighbours fused (tao_int4wo_decode_bf16):
    optional RMSNorm of x first; epilogue "none" -> [..., N], "swiglu" (rows interleaved
    (w1_i, w3_i)) -> [..., N/2], "rope_kv" with rope = (freqs, pos, k_cache, v_cache, n_head)
    -> rotated q [1, n_head, 1, D], k / v written into the caches at pos[0]."""
    _check(x, torch.bfloat16, "int4_decode x")
    N, K = packed.shape[0], x.shape[-1]
    if x.numel() != K:
        raise RuntimeError(f"int4_decode takes one token, got x of shape {tuple(x.shape)}")
    if norm_weight is not None:
        _check(norm_weight, torch.bfloat16, "int4_decode norm_weight")
        if not prologue_pays(N, K):  # normalise once in its own launch instead
            x, norm_weight = rmsnorm(x, norm_weight, eps), None
    epi = _EPILOGUES[epilogue]
    freqs = pos = kc = vc = None
    H = Hkv = D = T = 0
    if epi == 2:
        freqs, pos, kc, vc, H = rope
        _, Hkv, T, D = kc.shape
        y = torch.empty(1, H, 1, D, dtype=x.dtype, device=x.device)
    elif epi == 1:
        y = torch.empty(*x.shape[:-1], N // 2, dtype=x.dtype, device=x.device)
    else:
        y = torch.empty(*x.shape[:-1], N, dtype=x.dtype, device=x.device)
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    _lib.call("tao_int4wo_decode_bf16", x.data_ptr(), packed.data_ptr(), scale_and_zero.data_ptr(),
              N, K, int(group_size), ptr(norm_weight), float(eps), epi, y.data_ptr(), ptr(freqs),
              ptr(pos), ptr(kc), ptr(vc), H, Hkv, D, T, _stream(x))
    return y


def int8wo_decode(x: torch.Tensor, w: torch.Tensor, scale: torch.Tensor, norm_weight=None,
                  eps: float = 0.0, epilogue: str = "none", rope=None,
                  _entry: str = "tao_int8wo_decode_bf16") -> torch.Tensor:
    """One token through an int8 weight-only linear (w [N, K] int8, scale [N] bf16) with the
    int4_decode fusions (tao_int8wo_decode_bf16): optional RMSNorm of x; epilogue "none",
    "swiglu" or "rope_kv" as in int4_decode."""
    _check(x, torch.bfloat16, "int8wo_decode x")
    _check(w, torch.int8, "int8wo_decode w")
    N, K = w.shape
    if x.numel() != K:
        raise RuntimeError(f"int8wo_decode takes one token, got x of shape {tuple(x.shape)}")
    scale = scale.reshape(-1).contiguous()
    _check(scale, torch.bfloat16, "int8 decode scale")
    if scale.numel() != N:
        raise RuntimeError(f"int8 decode: {scale.numel()} scales for {N} rows")
    if norm_weight is not None:
        _check(norm_weight, torch.bfloat16, "int8wo_decode norm_weight")
    epi = _EPILOGUES[epilogue]
    freqs = pos = kc = vc = None
    H = Hkv = D = T = 0
    if epi == 2:
        freqs, pos, kc, vc, H = rope
        _, Hkv, T, D = kc.shape
        y = torch.empty(1, H, 1, D, dtype=x.dtype, device=x.device)
    elif epi == 1:
        y = torch.empty(*x.shape[:-1], N // 2, dtype=x.dtype, device=x.device)
    else:
        y = torch.empty(*x.shape[:-1], N, dtype=x.dtype, device=x.device)
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    _lib.call(_entry, x.data_ptr(), w.data_ptr(), scale.data_ptr(), N, K,
              ptr(norm_weight), float(eps), epi, y.data_ptr(), ptr(freqs), ptr(pos), ptr(kc),
              ptr(vc), H, Hkv, D, T, _stream(x))
    return y


def int8dq_decode(x: torch.Tensor, w: torch.Tensor, scale: torch.Tensor, norm_weight=None,
                  eps: float = 0.0, epilogue: str = "none", rope=None) -> torch.Tensor:
    """int8wo_decode for the int8 dynamic-activation linear (Int8DynamicActivationInt8Weight):
    the (normalised) token is quantised per token inside the kernel (tao_int8dq_decode_bf16)."""
    return int8wo_decode(x, w, scale, norm_weight, eps, epilogue, rope,
                         _entry="tao_int8dq_decode_bf16")


def argmax(logits: torch.Tensor) -> torch.Tensor:
    """bf16 logits [..., V] -> int64 [..., 1] index of the maximum (first on ties)."""
    _check(logits, torch.bfloat16, "argmax logits")
    out = torch.empty(*logits.shape[:-1], 1, dtype=torch.int64, device=logits.device)
    V = logits.shape[-1]
    _lib.call("tao_argmax_bf16", logits.data_ptr(), out.data_ptr(), logits.numel() // V, V,
              _stream(logits))
    return out


def argmax_advance(logits: torch.Tensor, cur: torch.Tensor, pos: torch.Tensor,
                   tokens: torch.Tensor) -> None:
    """Batch 1: cur[0, 0] = argmax(logits), tokens[0, pos + 1] = it, pos += 1, in one launch
    (tao_argmax_advance_bf16)."""
    _check(logits, torch.bfloat16, "argmax_advance logits")
    for t, n in ((cur, "cur"), (pos, "pos"), (tokens, "tokens")):
        _check(t, torch.int64, f"argmax_advance {n}")
    if cur.numel() != 1 or tokens.shape[0] != 1:
        raise RuntimeError("argmax_advance is batch 1")
    V = logits.shape[-1]
    _lib.call("tao_argmax_advance_bf16", logits.data_ptr(), V, cur.data_ptr(), pos.data_ptr(),
              tokens.data_ptr(), tokens.shape[1], _stream(logits))


def check_decode_status() -> None:
    """Raise if a decode kernel saw a KV-cache position outside the cache since the last check
    (tao_decode_status: the kernels skip that write instead of faulting; synchronous, so call it
    outside graph capture, e.g. after a generate())."""
    import ctypes

    bits = ctypes.c_int(0)
    _lib.call("tao_decode_status", ctypes.cast(ctypes.pointer(bits), ctypes.c_void_p))
    if bits.value & 1:
        raise RuntimeError("decode step at a position past the KV cache (max_seq_length): "
                           "no cache row was written; call setup_caches() with a larger "
                           "max_seq_length")
    if bits.value & 4:
        raise RuntimeError("a grouped (MoE) linear read an expert index outside [0, num_experts) "
                           "(clamped); those outputs are unspecified")
    if bits.value & 2:
        raise RuntimeError("a cross-workgroup hand-off (split-K reducer or fused decode "
                           "attention) timed out waiting for its producers; those outputs are "
                           "unspecified")
