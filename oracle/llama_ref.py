"""CPU oracle of the Llama decoder forward for BASELINE config 4 — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module (the product path never does). It restates the reference
gpt-fast model (torchao/_models/llama/model.py) over a plain dict of weights, entirely in fp32,
as the tolerance anchor for the quantized HIP decode path:

  RMSNorm            <- model.py:489-499 (x * rsqrt(mean(x^2) + eps), then * weight)
  rotary embedding   <- model.py:528-560 (pairs (x[2j], x[2j+1]) rotated by theta_j * pos;
                        the table is kept in fp32 here, the reference rounds it to bf16)
  attention block    <- model.py:417-475 (wqkv split q | k | v, GQA by repeat_interleave,
                        causal softmax attention, wo)
  feed-forward       <- model.py:478-486 (w2(silu(w1 x) * w3 x))
  block / model      <- model.py:397-414, 342-360 (pre-norm residual blocks, final norm, output)

Quantized weights enter as the reference CPU "dequant path" sees them: oracle.int4_qparams ->
int4_quantize -> int4_dequantize (bf16, bit-exact to the reference, tests/golden) -> fp32.
"""

import math
from typing import Dict

import torch

from oracle import oracle


def int4_dequant_weight(w_bf16: torch.Tensor, group_size: int) -> torch.Tensor:
    """bf16 [N, K] -> the reference's int4 tinygemm round trip (bf16), as fp32."""
    s, z = oracle.int4_qparams(w_bf16, group_size)
    q = oracle.int4_quantize(w_bf16, s, z, group_size)
    return oracle.int4_dequantize(q, s, z, group_size).float()


def rope_table(head_dim: int, base: float, seq_len: int) -> torch.Tensor:
    """[seq_len, head_dim/2, 2] (cos, sin) in fp64 -> fp32 (model.py:528-544)."""
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.float64)[: head_dim // 2]
                          / head_dim))
    ang = torch.outer(torch.arange(seq_len, dtype=torch.float64), inv)
    return torch.stack([ang.cos(), ang.sin()], dim=-1).float()


def _rope(x: torch.Tensor, tab: torch.Tensor) -> torch.Tensor:
    # x [S, H, D], tab [S, D/2, 2]  (model.py:547-560)
    xs = x.reshape(*x.shape[:-1], -1, 2)
    c, s = tab[:, None, :, 0], tab[:, None, :, 1]
    out = torch.stack([xs[..., 0] * c - xs[..., 1] * s, xs[..., 1] * c + xs[..., 0] * s], -1)
    return out.flatten(-2)


def _rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


@torch.no_grad()
def llama_forward_fp32(W: Dict[str, torch.Tensor], n_layer: int, n_head: int, n_kv: int,
                       rope_base: float, eps: float, tokens: torch.Tensor) -> torch.Tensor:
    """Causal forward of token ids [S] -> fp32 logits [S, vocab]. ``W`` holds fp32 tensors under
    the reference's parameter names (tok_embeddings.weight, layers.{i}.attention.wqkv.weight,
    ...wo.weight, ...feed_forward.{w1,w2,w3}.weight, ...{attention,ffn}_norm.weight,
    norm.weight, output.weight); linear weights already dequantized."""
    x = W["tok_embeddings.weight"][tokens]  # [S, dim]
    S, dim = x.shape
    D = dim // n_head
    tab = rope_table(D, rope_base, S)
    mask = torch.ones(S, S, dtype=torch.bool).tril()
    for i in range(n_layer):
        p = f"layers.{i}."
        h = _rmsnorm(x, W[p + "attention_norm.weight"], eps)
        qkv = h @ W[p + "attention.wqkv.weight"].t()
        q, k, v = qkv.split([n_head * D, n_kv * D, n_kv * D], dim=-1)
        q = _rope(q.view(S, n_head, D), tab).transpose(0, 1)  # [H, S, D]
        k = _rope(k.view(S, n_kv, D), tab).transpose(0, 1)
        v = v.view(S, n_kv, D).transpose(0, 1)
        rep = n_head // n_kv
        k, v = k.repeat_interleave(rep, 0), v.repeat_interleave(rep, 0)
        att = (q @ k.transpose(1, 2)) / math.sqrt(D)
        att = att.masked_fill(~mask, float("-inf")).softmax(-1)
        y = (att @ v).transpose(0, 1).reshape(S, n_head * D)
        x = x + y @ W[p + "attention.wo.weight"].t()
        h = _rmsnorm(x, W[p + "ffn_norm.weight"], eps)
        a = h @ W[p + "feed_forward.w1.weight"].t()
        b = h @ W[p + "feed_forward.w3.weight"].t()
        x = x + (torch.nn.functional.silu(a) * b) @ W[p + "feed_forward.w2.weight"].t()
    return _rmsnorm(x, W["norm.weight"], eps) @ W["output.weight"].t()
