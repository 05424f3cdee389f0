"""Multi-GPU (one process per GPU) sharding of the quantized linear path."""

from .colwise import (
    ColwiseShardedLinear,
    all_gather_columns,
    parallelize_colwise_,
    shard_linear_colwise,
)

__all__ = ["ColwiseShardedLinear", "all_gather_columns", "parallelize_colwise_", "shard_linear_colwise"]
