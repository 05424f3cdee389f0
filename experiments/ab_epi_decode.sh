#!/bin/bash
# Same-box A/B of the decode epilogue-operand prefetch: A = experiments/build/libold.so (before),
# B = experiments/build/libnew.so (after), alternated N times (default 3).
R=$(cd "$(dirname "$0")/.." && pwd)
N=${1:-3}
for i in $(seq "$N"); do
  for v in old new; do
    TORCHAO_MI355X_LIB="$R/experiments/build/lib$v.so" timeout -k 10 120 python3 "$R/experiments/ab_epi_decode.py" "$v" || exit 1
  done
done
