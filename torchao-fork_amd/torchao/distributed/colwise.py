"""Column (output-feature) sharding of linears over one process per GPU, RCCL all-gather.

SURVEY §8e. The reference gets tensor parallelism from DTensor in its tests only
(test/dtypes/test_affine_quantized_tensor_parallel.py:49-132: ``Shard(0)`` colwise weights,
replicated input, c10d all-gather). Here it is explicit and graph-capturable:

* rank r owns output rows ``[r N/P, (r+1) N/P)`` of W[N][K] (and of the bias);
* quantization is per row with groups along K, so sharding the bf16 weight and then quantizing
  the shard gives exactly the rows the full-model quantization would (no repacking, and each
  rank only ever materialises its own shard);
* forward: local linear (the gfx950 int4/int8 kernels via the AQT dispatch), then one
  ``all_gather_into_tensor`` of the bf16 output over the group (RCCL over xGMI with backend
  "nccl"; gloo for CPU tests), or no gather (``gather=False``) when a rowwise linear consumes
  the local columns (rowwise.py). Each output column is one row's dot product, computed by the
  same kernel math whatever P is, but the GEMV picks its launch shape (waves along K, rows per
  wave) from the local N, which can re-associate a column's fp32 sum: the gathered result
  agrees with the unsharded linear to one bf16 rounding (tests/test_gpu_configs.py, config 5),
  and is bit-identical wherever the shard's launch shape equals the full one.
"""

from typing import Callable, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["ColwiseShardedLinear", "shard_linear_colwise", "parallelize_colwise_"]


def _group_info(group):
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def shard_linear_colwise(linear: nn.Linear, rank: int, world: int) -> nn.Linear:
    """A new nn.Linear holding rows [rank N/P, (rank+1) N/P) of ``linear`` (N % P == 0)."""
    N, K = linear.out_features, linear.in_features
    if N % world:
        raise ValueError(f"out_features {N} is not divisible by the group size {world}")
    n = N // world
    rows = slice(rank * n, (rank + 1) * n)
    w = linear.weight
    shard = nn.Linear(K, n, bias=linear.bias is not None, device="meta")
    shard.weight = nn.Parameter(w.detach()[rows].clone(), requires_grad=False)
    if linear.bias is not None:
        shard.bias = nn.Parameter(linear.bias.detach()[rows].clone(), requires_grad=False)
    return shard


class ColwiseShardedLinear(nn.Module):
    """Wraps this rank's shard (``self.local``, an nn.Linear whose weight may be quantized)."""

    def __init__(self, local: nn.Linear, out_features: int, group=None,
                 local_fn: Optional[Callable] = None, gather: bool = True):
        super().__init__()
        self.local = local
        self.out_features = out_features
        self.in_features = local.in_features
        self.group = group
        self.gather = gather
        # local_fn(x, weight, bias) -> y_local; default F.linear (AQT dispatch -> HIP kernels)
        self.local_fn = local_fn or F.linear

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.local_fn(x, self.local.weight, self.local.bias)
        _, world = _group_info(self.group)
        if world == 1 or not self.gather:
            return y
        return all_gather_columns(y, self.out_features, self.group)

    def extra_repr(self):
        rank, world = _group_info(self.group)
        return f"in_features={self.in_features}, out_features={self.out_features}, shard={rank}/{world}"


def all_gather_columns(y_local: torch.Tensor, out_features: int, group=None) -> torch.Tensor:
    """[..., N/P] on every rank -> [..., N], ranks' column blocks in rank order."""
    _, world = _group_info(group)
    lead = y_local.shape[:-1]
    n = y_local.shape[-1]
    flat = y_local.reshape(-1, n).contiguous()
    M = flat.shape[0]
    if M == 1:  # rank blocks are already the output order
        out = torch.empty(world * n, dtype=y_local.dtype, device=y_local.device)
        dist.all_gather_into_tensor(out, flat.reshape(-1), group=group)
        return out.reshape(*lead, out_features)
    out = torch.empty(world * M, n, dtype=y_local.dtype, device=y_local.device)
    dist.all_gather_into_tensor(out, flat, group=group)  # rank blocks stacked along dim 0
    return out.view(world, M, n).permute(1, 0, 2).reshape(*lead, out_features)


def parallelize_colwise_(model: nn.Module, group=None,
                         filter_fn: Optional[Callable[[nn.Module, str], bool]] = None,
                         local_fn: Optional[Callable] = None) -> nn.Module:
    """Replace, in place, every selected nn.Linear by a ColwiseShardedLinear holding this rank's
    shard. Run it on the bf16 model, then ``quantize_`` the result: the inner shards quantize
    exactly as the full weights would."""
    rank, world = _group_info(group)
    filter_fn = filter_fn or (lambda m, fqn: isinstance(m, nn.Linear))

    def walk(mod: nn.Module, prefix: str):
        for name, child in list(mod.named_children()):
            fqn = f"{prefix}{name}"
            if isinstance(child, nn.Linear) and filter_fn(child, fqn):
                shard = shard_linear_colwise(child, rank, world)
                setattr(mod, name, ColwiseShardedLinear(shard, child.out_features, group, local_fn))
            elif not isinstance(child, ColwiseShardedLinear):
                walk(child, fqn + ".")

    walk(model, "")
    return model
