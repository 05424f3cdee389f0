"""Llama-family decoder for the end-to-end decode harness (BASELINE config 4).

Same module tree and parameter names as the reference's gpt-fast model
(torchao/_models/llama/model.py:243-501: ``tok_embeddings``, ``layers.{i}.attention.{wqkv,wo}``,
``layers.{i}.feed_forward.{w1,w2,w3}``, ``{attention,ffn}_norm``, ``norm``, ``output``), so
``quantize_`` filters and checkpoints keyed by those names apply unchanged. Every linear is a
plain ``nn.Linear``: after ``quantize_(model, Int4WeightOnlyConfig(...))`` its forward goes
through the AQT F.linear dispatch to the gfx950 HIP kernels.

Decode-time structure for one process per GPU and HIP graphs (no tracing compiler):
  * static KV cache [B, H_kv, T, D] per layer addressed by ``input_pos`` (a device tensor), so a
    decode step is graph-capturable and each replay advances by incrementing it in place;
  * ``enable_fused_kernels()`` (bf16, head_dim 128, GPU) switches one-token steps to the fused
    gfx950 kernels of csrc/decode_ops.hip: RMSNorm, RoPE + KV-cache write, flash-decoding
    attention, SiLU-mul, and the residual add folded into the wo / w2 linears as their bias
    (bf16(x + bf16(W a)) is exactly the bias epilogue at M = 1); with int4 weights the norms,
    RoPE + KV write and SwiGLU ride inside the wqkv / w13 / output GEMVs
    (tao_int4wo_decode_bf16) — 6 launches per layer;
  * fused prefill (S > 1 tokens): the linears on the MFMA GEMMs, RMSNorm, RoPE + KV-cache write
    and SiLU-mul on the same kernels (S rows each), ``F.scaled_dot_product_attention`` over the
    caches; ``prefill_next`` runs the output head at the last position only;
  * otherwise (CPU, or fused kernels off): torch ops, ``index_copy_`` into the caches, a
    causal-mask row gathered by ``input_pos``, ``F.scaled_dot_product_attention(enable_gqa=True)``;
  * rotary tables precomputed once (Llama-3.1 frequency scaling where configured).
"""

import math
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from torchao.utils import find_multiple

__all__ = ["ModelArgs", "Transformer", "KVCache", "llama_configs"]


@dataclass
class ModelArgs:
    block_size: int = 2048
    vocab_size: int = 32000
    n_layer: int = 32
    n_head: int = 32
    dim: int = 4096
    intermediate_size: Optional[int] = None
    n_local_heads: int = -1  # key/value heads (GQA); -1 = n_head
    head_dim: int = 0
    rope_base: float = 10000.0
    norm_eps: float = 1e-5
    rope_scaling: Optional[dict] = field(default=None)

    def __post_init__(self):
        if self.n_local_heads == -1:
            self.n_local_heads = self.n_head
        if self.intermediate_size is None:
            self.intermediate_size = find_multiple(int(2 * 4 * self.dim / 3), 256)
        self.head_dim = self.dim // self.n_head

    @classmethod
    def from_name(cls, name: str) -> "ModelArgs":
        """Exact config name, else the longest config name contained in ``name``
        (reference model.py:54-75 semantics: "Meta-Llama-3-8B" -> "Llama-3-8B")."""
        if name in llama_configs:
            return cls(**llama_configs[name])
        hits = sorted((k for k in llama_configs if k in name or k.upper() in name.upper()),
                      key=len, reverse=True)
        if not hits:
            raise ValueError(f"unknown model {name!r}; known: {sorted(llama_configs)}")
        return cls(**llama_configs[hits[0]])


_LLAMA31_SCALING = dict(factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0,
                        original_max_position_embeddings=8192)

# the reference's shapes (model.py:76-140) for the families the harness exercises
llama_configs = {
    "stories15M": dict(n_layer=6, n_head=6, dim=288),
    "stories110M": dict(n_layer=12, n_head=12, dim=768),
    "7B": dict(n_layer=32, n_head=32, dim=4096),
    "13B": dict(n_layer=40, n_head=40, dim=5120),
    "70B": dict(n_layer=80, n_head=64, dim=8192, n_local_heads=8, intermediate_size=28672),
    "Mistral-7B": dict(n_layer=32, n_head=32, n_local_heads=8, dim=4096,
                       intermediate_size=14336, vocab_size=32000),
    "Llama-3-8B": dict(block_size=8192, n_layer=32, n_head=32, n_local_heads=8, dim=4096,
                       intermediate_size=14336, vocab_size=128256, rope_base=500000),
    "Llama-3.1-8B": dict(block_size=131072, n_layer=32, n_head=32, n_local_heads=8, dim=4096,
                         intermediate_size=14336, vocab_size=128256, rope_base=500000,
                         rope_scaling=_LLAMA31_SCALING),
    "Llama-3-70B": dict(block_size=8192, n_layer=80, n_head=64, n_local_heads=8, dim=8192,
                        intermediate_size=28672, vocab_size=128256, rope_base=500000),
    "Llama-3.1-70B": dict(block_size=131072, n_layer=80, n_head=64, n_local_heads=8,
                          dim=8192, intermediate_size=28672, vocab_size=128256,
                          rope_base=500000, rope_scaling=_LLAMA31_SCALING),
}


class KVCache(nn.Module):
    """Static [B, H_kv, T, D] key/value buffers, updated in place at ``input_pos``."""

    def __init__(self, batch: int, seq_len: int, n_heads: int, head_dim: int, dtype, device=None):
        super().__init__()
        shape = (batch, n_heads, seq_len, head_dim)
        self.register_buffer("k_cache", torch.zeros(shape, dtype=dtype, device=device),
                             persistent=False)
        self.register_buffer("v_cache", torch.zeros(shape, dtype=dtype, device=device),
                             persistent=False)

    def update(self, input_pos: torch.Tensor, k: torch.Tensor, v: torch.Tensor):
        # k, v: [B, H_kv, S, D] at positions input_pos [S]
        self.k_cache.index_copy_(2, input_pos, k)
        self.v_cache.index_copy_(2, input_pos, v)
        return self.k_cache, self.v_cache


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return y.type_as(x) * self.weight


def _rope_freqs(cfg: ModelArgs, seq_len: int) -> torch.Tensor:
    """[seq_len, head_dim/2, 2] (cos, sin) in fp32; Llama-3.1 wavelength-dependent scaling."""
    d = cfg.head_dim
    inv = 1.0 / (cfg.rope_base ** (torch.arange(0, d, 2, dtype=torch.float64)[: d // 2] / d))
    sc = cfg.rope_scaling
    if sc is not None:
        old = sc["original_max_position_embeddings"]
        lo_wl = old / sc["low_freq_factor"]
        hi_wl = old / sc["high_freq_factor"]
        wl = 2 * torch.pi / inv
        lo_f, hi_f = sc["low_freq_factor"], sc["high_freq_factor"]
        smooth = (old / wl - lo_f) / (hi_f - lo_f)
        scaled = torch.where(wl > lo_wl, inv / sc["factor"], inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / sc["factor"] + smooth * inv, scaled)
    t = torch.arange(seq_len, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return torch.stack([ang.cos(), ang.sin()], dim=-1).float()


def _apply_rope(x: torch.Tensor, freqs: torch.Tensor) -> torch.Tensor:
    # x: [B, S, H, D] (pairs along D); freqs: [S, D/2, 2]
    xs = x.float().reshape(*x.shape[:-1], -1, 2)
    f = freqs.view(1, xs.size(1), 1, xs.size(3), 2)
    out = torch.stack([xs[..., 0] * f[..., 0] - xs[..., 1] * f[..., 1],
                       xs[..., 1] * f[..., 0] + xs[..., 0] * f[..., 1]], dim=-1)
    return out.flatten(3).type_as(x)


def kernels_rmsnorm(x: torch.Tensor, norm: "RMSNorm") -> torch.Tensor:
    from torchao._models.llama import kernels

    return kernels.rmsnorm(x, norm.weight, norm.eps)


def _linear_or_partials(x: torch.Tensor, lin: nn.Linear):
    """lin(x), or for an int4 linear the single-fetch GEMM's unreduced K-slice partials
    (kernels.PREFILL_PARTIALS) wrapped as ("partials", part) for _add_norm to sum."""
    from torchao._models.llama import kernels

    p4 = _int4_parts(lin) if kernels.PREFILL_PARTIALS else None
    if p4 is not None and x.dtype == torch.bfloat16:
        part = kernels.int4_linear_partials(x, *p4)
        if part is not None:
            return ("partials", part)
    return lin(x)


def _add_norm(x: torch.Tensor, pending, norm: "RMSNorm"):
    """(x + pending, RMSNorm(x + pending)) in one launch; pending is a bf16 linear output or
    _linear_or_partials' partials."""
    from torchao._models.llama import kernels

    if isinstance(pending, tuple):
        return kernels.add_rmsnorm_partials(x, pending[1], norm.weight, norm.eps)
    return kernels.add_rmsnorm(x, pending, norm.weight, norm.eps)


def _linear_plus(x: torch.Tensor, lin: nn.Linear, residual: torch.Tensor) -> torch.Tensor:
    """residual + lin(x); at one token the add rides on the linear's bias epilogue."""
    if x.numel() == x.shape[-1]:
        return F.linear(x, lin.weight, residual.reshape(-1))
    return residual + lin(x)


# Prefill: fold the SiLU-mul into the int4 w1||w3 GEMM's epilogue where a fused kernel serves the
# shape (tao_int4wo_linear_swiglu_bf16); False = the linear then tao_silu_mul_bf16.
PREFILL_SWIGLU = True
# Prefill: fold RoPE + the KV-cache write into the int4 wqkv GEMM's epilogue where a fused kernel
# serves the shape (tao_int4wo_linear_rope_kv_bf16); False = the linear then tao_rope_kv_bf16.
PREFILL_ROPE = True


def _int4_parts(lin: Optional[nn.Linear]):
    """(packed_weight, scale_and_zero, group_size) of an int4 weight-only linear on the gfx950
    row-stream layout (Int4WeightOnlyConfig), else None: the fused decode kernels read those
    operands directly."""
    w = getattr(lin, "weight", None)
    impl = getattr(w, "tensor_impl", None)
    packed = getattr(impl, "packed_weight", None)
    if packed is None or packed.dim() != 2 or not packed.is_cuda or lin.bias is not None:
        return None
    return packed, impl.scale_and_zero, w.block_size[-1]


def _int8wo_parts(lin: Optional[nn.Linear]):
    """(int_data [N, K] int8, scale [N]) of an int8 weight-only linear (Int8WeightOnlyConfig,
    PlainLayout) on the GPU, else None: the fused int8 decode kernels read those operands."""
    w = getattr(lin, "weight", None)
    if w is None or lin.bias is not None or not w.is_cuda:
        return None
    from torchao.dtypes.uintx.plain_layout import _linear_fp_act_int8_weight_check

    if not _linear_fp_act_int8_weight_check(torch.empty(0, dtype=torch.bfloat16), w, None):
        return None
    impl = w.tensor_impl
    # the fused kernels read bf16 per-row scales; anything else (fp32 scales of an fp32-quantized
    # weight) takes the regular linear, which casts them
    if impl.scale.dtype != torch.bfloat16 or impl.scale.numel() != impl.int_data.shape[0]:
        return None
    return impl.int_data, impl.scale.reshape(-1)


def _int8dq_parts(lin: Optional[nn.Linear]):
    """(int_data [N, K] int8, scale [N]) of an Int8DynamicActivationInt8WeightConfig linear with
    the default per-token activation recipe on the GPU, else None."""
    w = getattr(lin, "weight", None)
    if w is None or lin.bias is not None or not w.is_cuda:
        return None
    from torchao.quantization.linear_activation_quantized_tensor import (
        LinearActivationQuantizedTensor,
    )
    from torchao.quantization.quant_api import _int8_symm_per_token_reduced_range_quant

    if not (isinstance(w, LinearActivationQuantizedTensor) and not w.quant_kwargs
            and w.input_quant_func is _int8_symm_per_token_reduced_range_quant):
        return None
    # the weight criteria of the one-token int8-dyn dispatch (_fused_int8_dyn_decode)
    from torchao.dtypes.affine_quantized_tensor import AffineQuantizedTensor
    from torchao.dtypes.uintx.plain_layout import PlainLayout, _aqt_is_int8

    inner = w.original_weight_tensor
    if not (isinstance(inner, AffineQuantizedTensor) and _aqt_is_int8(inner)
            and inner.dtype == torch.bfloat16 and isinstance(inner._layout, PlainLayout)
            and len(inner.shape) == 2 and inner.tensor_impl.int_data.is_cuda):
        return None
    return inner.tensor_impl.int_data, inner.tensor_impl.scale.reshape(-1)


def _fused_decode(x, lin, norm=None, epilogue="none", rope=None):
    """One token through ``lin`` with the decode fusions, on whichever fused kernel its weight
    format has (int4 weight-only, int8 weight-only); None if neither applies."""
    from torchao._models.llama import kernels

    if x.numel() != x.shape[-1]:
        return None
    nw = None if norm is None else norm.weight
    eps = 0.0 if norm is None else norm.eps
    p4 = _int4_parts(lin)
    if p4 is not None:
        return kernels.int4_decode(x, *p4, norm_weight=nw, eps=eps, epilogue=epilogue, rope=rope)
    p8 = _int8wo_parts(lin)
    if p8 is not None:
        return kernels.int8wo_decode(x, *p8, norm_weight=nw, eps=eps, epilogue=epilogue, rope=rope)
    pq = _int8dq_parts(lin)
    if pq is not None and (nw is None or x.shape[-1] <= 8192):
        return kernels.int8dq_decode(x, *pq, norm_weight=nw, eps=eps, epilogue=epilogue, rope=rope)
    return None


class Attention(nn.Module):
    def __init__(self, cfg: ModelArgs):
        super().__init__()
        self.n_head, self.n_kv, self.head_dim = cfg.n_head, cfg.n_local_heads, cfg.head_dim
        qkv = (cfg.n_head + 2 * cfg.n_local_heads) * cfg.head_dim
        self.wqkv = nn.Linear(cfg.dim, qkv, bias=False)
        self.wo = nn.Linear(cfg.dim, cfg.dim, bias=False)
        self.kv_cache: Optional[KVCache] = None

    def forward(self, x, freqs, mask, input_pos):
        B, S, _ = x.shape
        q_sz, kv_sz = self.n_head * self.head_dim, self.n_kv * self.head_dim
        q, k, v = self.wqkv(x).split([q_sz, kv_sz, kv_sz], dim=-1)
        q = _apply_rope(q.view(B, S, self.n_head, self.head_dim), freqs)
        k = _apply_rope(k.view(B, S, self.n_kv, self.head_dim), freqs)
        v = v.view(B, S, self.n_kv, self.head_dim)
        q, k, v = (t.transpose(1, 2) for t in (q, k, v))
        if self.kv_cache is not None:
            k, v = self.kv_cache.update(input_pos, k, v)
        y = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, enable_gqa=True)
        return self.wo(y.transpose(1, 2).reshape(B, S, q_sz))

    def forward_prefill(self, x, freqs_table, mask, input_pos, wo=True):
        """S > 1 tokens on the gfx950 kernels: wqkv (MFMA GEMM), RoPE + KV-cache write in one
        launch, then F.scaled_dot_product_attention over the caches (forward's math). wo=False:
        the attention output [B, S, H * D] before the wo linear."""
        from torchao._models.llama import kernels

        B, S, _ = x.shape
        kv = self.kv_cache
        q = None
        p4 = _int4_parts(self.wqkv) if PREFILL_ROPE else None
        if p4 is not None and x.is_contiguous():  # wqkv GEMM with RoPE + KV write (one launch)
            q = kernels.int4_linear_rope_kv(x, *p4, freqs_table, input_pos, kv.k_cache,
                                            kv.v_cache, self.n_head)
        if q is None:
            q = kernels.rope_kv(self.wqkv(x), freqs_table, input_pos, kv.k_cache, kv.v_cache,
                                self.n_head)
        if kernels.PREFILL_ATTN and self.head_dim == 128 and q.dtype == torch.bfloat16:
            # the causal mask over the caches is keys 0..input_pos[s] for query s
            y = kernels.attn_prefill(q, kv.k_cache, kv.v_cache, input_pos,
                                     1.0 / math.sqrt(self.head_dim))
            return self.wo(y) if wo else y
        y = F.scaled_dot_product_attention(q, kv.k_cache, kv.v_cache, attn_mask=mask,
                                           enable_gqa=True)
        y = y.transpose(1, 2).reshape(B, S, self.n_head * self.head_dim)
        return self.wo(y) if wo else y

    def prefill_last(self, x, freqs_table, input_pos):
        """forward_prefill's q / K / V for every row (the KV caches need them all), then the
        attention of the LAST query only -> [B, 1, H * D] (the greedy prefill's last block)."""
        from torchao._models.llama import kernels

        kv = self.kv_cache
        q = None
        p4 = _int4_parts(self.wqkv) if PREFILL_ROPE else None
        if p4 is not None and x.is_contiguous():
            q = kernels.int4_linear_rope_kv(x, *p4, freqs_table, input_pos, kv.k_cache,
                                            kv.v_cache, self.n_head)
        if q is None:
            q = kernels.rope_kv(self.wqkv(x), freqs_table, input_pos, kv.k_cache, kv.v_cache,
                                self.n_head)
        return kernels.attn_decode(q[:, :, -1:].contiguous(), kv.k_cache, kv.v_cache,
                                   input_pos[-1:], 1.0 / math.sqrt(self.head_dim))

    def forward_fused(self, x, freqs_table, input_pos, residual, norm=None):
        from torchao._models.llama import kernels

        kv = self.kv_cache
        scale = 1.0 / math.sqrt(self.head_dim)
        # int4 at batch 1: RMSNorm -> wqkv -> RoPE + KV write -> attention in one launch
        pq = None if (norm is None or not kernels.DECODE_QKV_ATTN) else _int4_parts(self.wqkv)
        if (pq is not None and x.numel() == x.shape[-1] and kv.k_cache.shape[0] == 1
                and kv.k_cache.shape[2] <= kernels.QKV_ATTN_MAX_T
                and kernels.prologue_pays(pq[0].shape[0], x.shape[-1])
                and kernels.qkv_attn_supported(pq[0].shape[0], x.shape[-1], self.n_head,
                                               kv.k_cache.shape[1], self.head_dim)):
            y = kernels.int4_qkv_attn(x, *pq, norm.weight, norm.eps, freqs_table, input_pos,
                                      kv.k_cache, kv.v_cache, self.n_head, scale)
            return _linear_plus(y, self.wo, residual)
        # RMSNorm -> wqkv -> RoPE + KV-cache write in one launch (int4 / int8 weight-only)
        q = None if norm is None else _fused_decode(
            x, self.wqkv, norm, "rope_kv", (freqs_table, input_pos, kv.k_cache, kv.v_cache,
                                            self.n_head))
        if q is None:
            if norm is not None:
                x = kernels.rmsnorm(x, norm.weight, norm.eps)
            q = kernels.rope_kv(self.wqkv(x), freqs_table, input_pos, kv.k_cache, kv.v_cache,
                                self.n_head)
        # int4 wo at batch 1: the attention split over key ranges (more workgroups than heads),
        # its merge folded into wo's x load (one launch each, as the unsplit pair)
        p4 = _int4_parts(self.wo)
        T = kv.k_cache.shape[2]
        if (p4 is not None and kernels.ATTN_SPLITS and q.shape[0] == 1 and self.head_dim == 128
                and kernels.ATTN_SPLIT_MIN_T <= T <= kernels.ATTN_SPLIT_MAX_T):
            part = kernels.attn_decode_split(q, kv.k_cache, kv.v_cache, input_pos, scale,
                                             kernels.ATTN_SPLITS)
            return kernels.int4_attn_out(part, self.n_head, *p4, residual=residual)
        y = kernels.attn_decode(q, kv.k_cache, kv.v_cache, input_pos, scale)
        return _linear_plus(y, self.wo, residual)


class FeedForward(nn.Module):
    def __init__(self, cfg: ModelArgs):
        super().__init__()
        self.w1 = nn.Linear(cfg.dim, cfg.intermediate_size, bias=False)
        self.w3 = nn.Linear(cfg.dim, cfg.intermediate_size, bias=False)
        self.w2 = nn.Linear(cfg.intermediate_size, cfg.dim, bias=False)
        self.w13: Optional[nn.Linear] = None

    def fuse_w13(self):
        """Merge w1 and w3 (same input) into one [2I, dim] linear: one weight stream and one
        launch per token instead of two. Rows interleave (w1_0, w3_0, w1_1, w3_1, ...) so
        each gate / up pair lands in adjacent outputs, which is what the SwiGLU epilogue of
        the fused int4 decode kernel and the pair mode of silu_mul read. Row-wise quantization
        makes quantizing the merged weight identical to quantizing w1 and w3 apart, so fuse
        before or after loading."""
        w = torch.stack([self.w1.weight.detach(), self.w3.weight.detach()], dim=1).flatten(0, 1)
        self.w13 = nn.Linear(w.shape[1], w.shape[0], bias=False, device="meta")
        self.w13.weight = nn.Parameter(w, requires_grad=False)
        del self.w1, self.w3
        self.w1 = self.w3 = None

    def _gate_up(self, x):
        if self.w13 is None:
            return self.w1(x), self.w3(x)
        h = self.w13(x).unflatten(-1, (-1, 2))
        return h[..., 0], h[..., 1]

    def forward(self, x):
        a, b = self._gate_up(x)
        return self.w2(F.silu(a) * b)

    def swiglu_prefill(self, x):
        """silu(w1 x) * w3 x for S > 1 tokens on the gfx950 kernels: the int4 w1||w3 GEMM with the
        SiLU-mul in its epilogue where a fused kernel serves the shape, else the linear(s) and
        tao_silu_mul_bf16."""
        from torchao._models.llama import kernels

        p4 = _int4_parts(self.w13) if (self.w13 is not None and PREFILL_SWIGLU) else None
        if p4 is not None:
            g = kernels.int4_linear_swiglu(x, *p4)
            if g is not None:
                return g
        if self.w13 is not None:
            return kernels.silu_mul(self.w13(x))
        return kernels.silu_mul(self.w1(x), self.w3(x))

    def forward_fused(self, x, residual, norm=None):
        from torchao._models.llama import kernels

        if (kernels.DECODE_FFN_ENGINE and norm is not None and self.w13 is not None
                and x.numel() == x.shape[-1] and residual is x):
            p13, p2 = _int4_parts(self.w13), _int4_parts(self.w2)
            if (p13 is not None and p2 is not None and p13[2] == p2[2]
                    and kernels.ffn_engine_supported(x.shape[-1], p13[0].shape[0] // 2, p13[2])):
                return kernels.int4_ffn_engine(x, norm.weight, norm.eps, p13, p2)
        if norm is not None:
            # RMSNorm -> w13 -> SwiGLU in one launch (int4 / int8 weight-only)
            g = None if self.w13 is None else _fused_decode(x, self.w13, norm, "swiglu")
            if g is not None:
                return _linear_plus(g, self.w2, residual)
            x = kernels.rmsnorm(x, norm.weight, norm.eps)
        if self.w13 is not None:
            g = kernels.silu_mul(self.w13(x))
        else:
            g = kernels.silu_mul(self.w1(x), self.w3(x))
        return _linear_plus(g, self.w2, residual)


class TransformerBlock(nn.Module):
    def __init__(self, cfg: ModelArgs):
        super().__init__()
        self.attention = Attention(cfg)
        self.feed_forward = FeedForward(cfg)
        self.attention_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.ffn_norm = RMSNorm(cfg.dim, cfg.norm_eps)

    def forward(self, x, freqs, mask, input_pos):
        h = x + self.attention(self.attention_norm(x), freqs, mask, input_pos)
        return h + self.feed_forward(self.ffn_norm(h))

    def forward_fused(self, x, freqs_table, input_pos):
        h = self.attention.forward_fused(x, freqs_table, input_pos, x, self.attention_norm)
        return self.feed_forward.forward_fused(h, h, self.ffn_norm)

    def forward_prefill(self, x, freqs_table, mask, input_pos):
        """forward() for S > 1 tokens with the norms, RoPE + KV write and SiLU-mul on the
        gfx950 kernels (one launch each instead of ~8, ~20 and 2 eager torch ops)."""
        from torchao._models.llama import kernels

        an, fn = self.attention_norm, self.ffn_norm
        h = x + self.attention.forward_prefill(kernels.rmsnorm(x, an.weight, an.eps), freqs_table,
                                               mask, input_pos)
        ff = self.feed_forward
        xn = kernels.rmsnorm(h, fn.weight, fn.eps)
        return h + ff.w2(ff.swiglu_prefill(xn))


class Transformer(nn.Module):
    def __init__(self, cfg: ModelArgs):
        super().__init__()
        self.config = cfg
        self.tok_embeddings = nn.Embedding(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList(TransformerBlock(cfg) for _ in range(cfg.n_layer))
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.output = nn.Linear(cfg.dim, cfg.vocab_size, bias=False)
        self.max_batch = self.max_seq = -1
        self.fused = False

    @classmethod
    def from_name(cls, name: str) -> "Transformer":
        return cls(ModelArgs.from_name(name))

    def setup_caches(self, max_batch_size: int, max_seq_length: int):
        """Allocate the static KV caches, rotary table and causal mask on the model's device."""
        cfg = self.config
        max_seq_length = find_multiple(max_seq_length, 8)
        if self.max_batch >= max_batch_size and self.max_seq >= max_seq_length:
            return
        self.max_batch, self.max_seq = max_batch_size, max_seq_length
        dev = self.norm.weight.device
        dtype = self.norm.weight.dtype
        for blk in self.layers:
            blk.attention.kv_cache = KVCache(max_batch_size, max_seq_length, cfg.n_local_heads,
                                             cfg.head_dim, dtype, dev)
        self.register_buffer("freqs", _rope_freqs(cfg, cfg.block_size).to(dev), persistent=False)
        mask = torch.tril(torch.ones(max_seq_length, max_seq_length, dtype=torch.bool, device=dev))
        self.register_buffer("causal_mask", mask, persistent=False)

    def fuse_w13(self) -> "Transformer":
        for blk in self.layers:
            blk.feed_forward.fuse_w13()
        return self

    def enable_fused_kernels(self, enable: bool = True) -> bool:
        """Route one-token steps through the fused gfx950 decode kernels (bf16 activations,
        head_dim 128, GPU). Returns whether they are on."""
        cfg = self.config
        ok = (self.norm.weight.is_cuda and self.norm.weight.dtype == torch.bfloat16
              and cfg.head_dim == 128 and cfg.n_head % cfg.n_local_heads == 0
              and cfg.n_head // cfg.n_local_heads in (1, 2, 4, 8) and cfg.dim % 8 == 0)
        self.fused = bool(enable and ok)
        return self.fused

    def _forward_fused(self, idx: torch.Tensor, input_pos: torch.Tensor) -> torch.Tensor:
        """One token per sequence through the fused kernels -> bf16 logits [B, 1, vocab]."""
        from torchao._models.llama import kernels

        x = self.tok_embeddings(idx)
        for blk in self.layers:
            x = blk.forward_fused(x, self.freqs, input_pos)
        return self._head_fused(x)

    def _head_fused(self, x: torch.Tensor) -> torch.Tensor:
        from torchao._models.llama import kernels

        y = _fused_decode(x, self.output, self.norm)  # final RMSNorm inside the head GEMV
        if y is not None:
            return y
        return self.output(kernels.rmsnorm(x, self.norm.weight, self.norm.eps))

    def _layers_prefill(self, idx: torch.Tensor, input_pos: torch.Tensor,
                        last_only: bool = False) -> torch.Tensor:
        """The blocks over S > 1 tokens -> hidden states [B, S, dim]; last_only (greedy prefill,
        kernels.PREFILL_LAST_ROW): [B, 1, dim] of the last position, the last block past its
        wqkv run on the one-token kernels."""
        from torchao._models.llama import kernels

        mask = self.causal_mask[None, None, input_pos]  # [1, 1, S, T]
        x = self.tok_embeddings(idx)
        last_only = (last_only and kernels.PREFILL_LAST_ROW and kernels.PREFILL_ADD_NORM
                     and self.config.head_dim == 128 and x.dtype == torch.bfloat16)
        if not kernels.PREFILL_ADD_NORM:
            for blk in self.layers:
                x = blk.forward_prefill(x, self.freqs, mask, input_pos)
            return x
        # each residual add fused with the RMSNorm that follows it (tao_add_rmsnorm_bf16): the
        # w2 output of block i is added at block i + 1's attention norm, the last one at the end
        pending = None
        for i, blk in enumerate(self.layers):
            an, fn, ff = blk.attention_norm, blk.ffn_norm, blk.feed_forward
            if pending is None:
                xn = kernels.rmsnorm(x, an.weight, an.eps)
            else:
                x, xn = _add_norm(x, pending, an)
            if last_only and i == len(self.layers) - 1:
                y = blk.attention.prefill_last(xn, self.freqs, input_pos)
                h = _linear_plus(y, blk.attention.wo, x[:, -1:].contiguous())
                return ff.forward_fused(h, h, fn)
            y = blk.attention.forward_prefill(xn, self.freqs, mask, input_pos, wo=False)
            x, hn = _add_norm(x, _linear_or_partials(y, blk.attention.wo), fn)
            pending = _linear_or_partials(ff.swiglu_prefill(hn), ff.w2)
        if pending is None:
            return x
        if isinstance(pending, tuple):  # the last w2's partials: h only (its norm is unused)
            return _add_norm(x, pending, self.norm)[0]
        return x + pending

    def prefill_next(self, idx: torch.Tensor, input_pos: torch.Tensor) -> torch.Tensor:
        """Greedy next token [B, 1] after the prompt ``idx`` [B, S] (the reference's prefill:
        logits[:, -1].argmax). On the fused path only the last position goes through the output
        head (one M = 1 launch per row instead of an M = S GEMM over the 128K vocabulary)."""
        if not (self.fused and idx.shape[1] > 1):
            return self(idx, input_pos)[:, -1].argmax(dim=-1, keepdim=True).to(idx.dtype)
        from torchao._models.llama import kernels

        x = self._layers_prefill(idx, input_pos, last_only=True)[:, -1:].contiguous()  # [B, 1, dim]
        return kernels.argmax(self._head_fused(x)[:, -1]).to(idx.dtype)

    def decode_next(self, idx: torch.Tensor, input_pos: torch.Tensor) -> torch.Tensor:
        """Greedy next token [B, 1] for one token per sequence; on the fused path the argmax
        runs on the bf16 logits (the same maximum as on their fp32 image, no conversion)."""
        if self.fused and idx.shape[1] == 1:
            from torchao._models.llama import kernels

            return kernels.argmax(self._forward_fused(idx, input_pos)[:, -1]).to(idx.dtype)
        return self(idx, input_pos)[:, -1].argmax(dim=-1, keepdim=True).to(idx.dtype)

    def decode_advance(self, cur: torch.Tensor, pos: torch.Tensor, tokens: torch.Tensor) -> bool:
        """Graph decode step for batch 1 on the fused path: the token in ``cur`` at position
        ``pos`` through the model, then one kernel takes the greedy next token into ``cur`` and
        ``tokens[0, pos + 1]`` and advances ``pos``. Returns False (nothing done) off that path."""
        if not (self.fused and cur.shape == (1, 1) and tokens.shape[0] == 1):
            return False
        from torchao._models.llama import kernels

        kernels.argmax_advance(self._forward_fused(cur, pos)[:, -1], cur, pos, tokens)
        return True

    def forward(self, idx: torch.Tensor, input_pos: torch.Tensor) -> torch.Tensor:
        """idx [B, S] token ids at positions input_pos [S] -> logits [B, S, vocab] (fp32)."""
        assert self.max_seq > 0, "call setup_caches() first"
        if self.fused and idx.shape[1] == 1:
            return self._forward_fused(idx, input_pos).float()
        if self.fused:
            x = self._layers_prefill(idx, input_pos)
            return self.output(kernels_rmsnorm(x, self.norm)).float()
        mask = self.causal_mask[None, None, input_pos]  # [1, 1, S, T]
        freqs = self.freqs[input_pos]
        x = self.tok_embeddings(idx)
        for blk in self.layers:
            x = blk(x, freqs, mask, input_pos)
        return self.output(self.norm(x)).float()
