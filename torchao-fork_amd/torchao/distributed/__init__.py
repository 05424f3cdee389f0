"""Multi-GPU (one process per GPU) sharding of the quantized linear path: colwise shards with an
RCCL all-gather, rowwise shards with an all-reduce, and their Megatron pairing."""

from .colwise import (
    ColwiseShardedLinear,
    all_gather_columns,
    parallelize_colwise_,
    shard_linear_colwise,
)
from .rowwise import (
    RowwiseShardedLinear,
    all_reduce_partial,
    shard_linear_rowwise,
    shard_rows,
    shard_wqkv_by_heads,
)

__all__ = ["ColwiseShardedLinear", "all_gather_columns", "parallelize_colwise_",
           "shard_linear_colwise", "RowwiseShardedLinear", "all_reduce_partial",
           "shard_linear_rowwise", "shard_rows", "shard_wqkv_by_heads"]
