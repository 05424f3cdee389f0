#!/bin/bash
# The decode GEMVs' RMSNorm prologue under timing-only variant builds (experiments/variant.sh:
# normdbg1 = no cross-wave exchange, normdbg2 = exchange kept, x stored unnormalised), two passes
# of experiments/bench_decode.py each. GPU-box step: bash experiments/norm_variants.sh TAG
cd "$(dirname "$0")/.." || exit 1
export PYTHONPATH=torchao-fork_amd:experiments TMPDIR=/tmp
O=gpurun_out/$1.jsonl
: > $O
for pass in 1 2; do
  for v in shipped normdbg1 normdbg2; do
    lib=""
    [ "$v" != shipped ] && lib=experiments/build/libvar_$v.so
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $O
    TORCHAO_MI355X_LIB=$lib timeout -k 10 200 python -u experiments/bench_decode.py >> $O \
      2>> gpurun_out/$1.err || exit $?
  done
done
cat $O
