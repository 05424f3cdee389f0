#!/bin/bash
# A/B of the e2e decode harness between an alternative library build (A) and the in-tree one
# (B), alternating runs on the same box: bash experiments/ab_e2e.sh LIB_A QUANT ROUNDS
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
LIBA=$1; Q=${2:-int4wo-32}; N=${3:-2}
cd "$R/torchao-fork_amd"
for i in $(seq "$N"); do
  for v in A B; do
    if [ "$v" = A ]; then export TORCHAO_MI355X_LIB="$LIBA"; else unset TORCHAO_MI355X_LIB; fi
    out=$(timeout -k 10 200 python3 -m torchao._models.llama.generate -q "$Q" --num_samples 3 2>/dev/null)
    echo "$v $(echo "$out" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["quantization"], d["decode_tokens_per_s"], d["decode_ms_per_token"], d["prefill_ms"])')"
  done
done
