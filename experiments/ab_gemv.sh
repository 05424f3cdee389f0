#!/bin/bash
# A/B of the int4 GEMV between an alternative library build (A) and the in-tree one (B) on the
# same box, alternating: per-shape graph timings (probe_graph_shapes.py) and the bench step.
# usage: bash experiments/ab_gemv.sh LIB_A ROUNDS
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
LIBA=$1; N=${2:-2}
for i in $(seq "$N"); do
  for v in A B; do
    if [ "$v" = A ]; then export TORCHAO_MI355X_LIB="$LIBA"; else unset TORCHAO_MI355X_LIB; fi
    timeout -k 10 120 python3 "$R/experiments/probe_graph_shapes.py" 2>/dev/null | sed "s/^/$v /"
    timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-reference-gpu --no-prefill \
      2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v bench', d['value'], d['roofline']['kernel_ms_per_step'])"
  done
done
