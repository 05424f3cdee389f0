#!/bin/bash
# A/B of the e2e decode harness between generate.py argument sets, alternating runs on the same
# box: bash experiments/ab_e2e_args.sh ROUNDS QUANT "ARGS_A" "ARGS_B" ["ARGS_C" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; Q=$2; shift 2
cd "$R/torchao-fork_amd"
for i in $(seq "$N"); do
  for a in "$@"; do
    out=$(timeout -k 10 200 python3 -m torchao._models.llama.generate -q "$Q" --num_samples 3 $a 2>/dev/null)
    echo "{\"args\": \"$a\", \"result\": $(echo "$out" | tail -1)}"
  done
done
