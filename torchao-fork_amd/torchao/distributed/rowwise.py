"""Row (input-feature) sharding and the Megatron colwise -> rowwise pairing, over one process per
GPU (RCCL all-reduce over xGMI with backend "nccl"; gloo for the CPU tests).

The reference's tensor-parallel test (test/dtypes/test_affine_quantized_tensor_parallel.py:49-80,
120-132) slices the *quantized* up projection by output rows (``Shard(0)``, colwise) and the down
projection by input columns (``Shard(1)``, rowwise), feeds the colwise output to the rowwise
linear without gathering it, and sums the rowwise partial outputs with one all-reduce. Here:

* a rowwise shard of W[N][K] is the column block ``[r K/P, (r+1) K/P)``; int4 / int8 weights are
  quantized per row with groups along K, so when K/P is a multiple of the group size the shard's
  (q, scale, zero) are exactly the full quantization's columns (shard-then-quantize ==
  quantize-then-slice) and no repacking happens;
* forward: local linear on this rank's slice of the input (the colwise predecessor's local
  output), one ``all_reduce(SUM)`` of the [..., N] partial, then the bias once. The partials are
  the local linear's bf16 outputs, as the reference's DTensor path reduces them; the sum matches
  the unsharded linear to bf16 rounding, not bit for bit;
* a Llama block pairs wqkv (colwise by attention heads: q, k and v heads of this rank) with wo
  (rowwise) and w1 || w3 (colwise) with w2 (rowwise): two all-reduces per layer instead of one
  gather per linear.
"""

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from .colwise import _group_info

__all__ = ["RowwiseShardedLinear", "shard_linear_rowwise", "shard_wqkv_by_heads",
           "shard_rows", "all_reduce_partial"]


def shard_rows(linear: nn.Linear, rows: torch.Tensor) -> nn.Linear:
    """A new nn.Linear holding the given output rows (index tensor) of ``linear``."""
    K = linear.in_features
    shard = nn.Linear(K, rows.numel(), bias=linear.bias is not None, device="meta")
    shard.weight = nn.Parameter(linear.weight.detach()[rows].clone(), requires_grad=False)
    if linear.bias is not None:
        shard.bias = nn.Parameter(linear.bias.detach()[rows].clone(), requires_grad=False)
    return shard


def shard_wqkv_by_heads(wqkv: nn.Linear, n_head: int, n_kv: int, head_dim: int, rank: int,
                        world: int) -> nn.Linear:
    """Colwise shard of a fused [q | k | v] projection by heads: this rank's H/P query heads,
    then its Hkv/P key heads, then its Hkv/P value heads (rows of the reference layout
    model.py:417-470), so local attention runs on whole heads."""
    if n_head % world or n_kv % world:
        raise ValueError(f"heads ({n_head} q, {n_kv} kv) not divisible by the group size {world}")
    hq, hk = n_head // world, n_kv // world
    q0 = rank * hq * head_dim
    k0 = n_head * head_dim + rank * hk * head_dim
    v0 = (n_head + n_kv) * head_dim + rank * hk * head_dim
    rows = torch.cat([torch.arange(q0, q0 + hq * head_dim), torch.arange(k0, k0 + hk * head_dim),
                      torch.arange(v0, v0 + hk * head_dim)])
    return shard_rows(wqkv, rows)


def shard_linear_rowwise(linear: nn.Linear, rank: int, world: int,
                         group_size: Optional[int] = None) -> nn.Linear:
    """A new bias-free nn.Linear holding input columns [rank K/P, (rank+1) K/P) of ``linear``
    (K % P == 0, and K/P % group_size == 0 when given). The bias stays with the
    RowwiseShardedLinear and is added once, after the reduction."""
    N, K = linear.out_features, linear.in_features
    if K % world:
        raise ValueError(f"in_features {K} is not divisible by the group size {world}")
    k = K // world
    if group_size and k % group_size:
        raise ValueError(f"K/P = {k} is not a multiple of the quantization group {group_size}")
    shard = nn.Linear(k, N, bias=False, device="meta")
    shard.weight = nn.Parameter(linear.weight.detach()[:, rank * k:(rank + 1) * k].clone(),
                                requires_grad=False)
    return shard


def all_reduce_partial(y: torch.Tensor, group=None) -> torch.Tensor:
    """Sum a [..., N] partial output over the group (in place on a contiguous copy)."""
    _, world = _group_info(group)
    if world == 1:
        return y
    y = y.contiguous()
    dist.all_reduce(y, op=dist.ReduceOp.SUM, group=group)
    return y


class RowwiseShardedLinear(nn.Module):
    """This rank's input-column shard (``self.local``, weight possibly quantized) + all-reduce.

    ``forward(x_local)`` takes the rank's [..., K/P] slice of the input, i.e. the un-gathered
    output of a colwise predecessor; ``forward_full(x)`` slices a replicated input first."""

    def __init__(self, local: nn.Linear, in_features: int, bias: Optional[torch.Tensor] = None,
                 group=None):
        super().__init__()
        self.local = local
        self.in_features = in_features
        self.out_features = local.out_features
        self.group = group
        self.bias = None if bias is None else nn.Parameter(bias.detach().clone(),
                                                           requires_grad=False)

    def forward(self, x_local: torch.Tensor) -> torch.Tensor:
        y = all_reduce_partial(F.linear(x_local, self.local.weight), self.group)
        return y if self.bias is None else y + self.bias

    def forward_full(self, x: torch.Tensor) -> torch.Tensor:
        rank, world = _group_info(self.group)
        k = self.in_features // world
        return self.forward(x[..., rank * k:(rank + 1) * k])

    def extra_repr(self):
        rank, world = _group_info(self.group)
        return (f"in_features={self.in_features}, out_features={self.out_features}, "
                f"shard={rank}/{world}")
