#!/bin/bash
# e2e decode harness (config 4) alternated between the in-tree library and LIB_B on one box:
#   bash experiments/ab_lib_e2e.sh TAG LIB_B [ROUNDS]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1.jsonl
: > $O
for i in $(seq "${3:-2}"); do
  for lib in "" "$2"; do
    out=$(cd torchao-fork_amd && TORCHAO_MI355X_LIB=${lib:+../$lib} timeout -k 10 200 python3 -m \
      torchao._models.llama.generate -q int4wo-32 --num_samples 5 2>>../gpurun_out/$1.err) || exit $?
    echo "{\"lib\": \"${lib:-shipped}\", \"result\": $(echo "$out" | tail -1)}" >> $O
  done
done
python3 - "$O" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line); r = d["result"]
    print(d["lib"], r["decode_tokens_per_s"], r["prefill_ms"], r["graph_eager_token_match"])
PY
