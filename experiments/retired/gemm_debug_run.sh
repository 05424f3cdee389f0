#!/bin/bash
# Time the prefill GEMM configurations on every TAO_GEMM_DEBUG variant (gemm_debug.sh build first).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for cfg in "int4 128 4096 4096" "int4 128 28672 4096" "int8dyn 128 4096 4096" "int8dyn 128 28672 4096"; do
  bash "$R/experiments/gemm_debug.sh" run $cfg 0 0 0 40
done
