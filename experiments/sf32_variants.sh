#!/bin/bash
# w1||w3 (int4 M=128 28672x4096, 128-column tiles, one split) timed under each timing-only variant
# library built by experiments/variant.sh, loader waves off (1) and on (2), two passes; then the
# per-step stamps (libvar_steps). GPU-box step: bash experiments/sf32_variants.sh TAG VAR...
cd "$(dirname "$0")/.." || exit 1
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/$tag.jsonl
: > $O
for pass in 1 2; do
  for v in shipped "$@"; do
    lib=""
    [ "$v" != shipped ] && lib=experiments/build/libvar_$v.so
    for ld in 1 2; do
      TORCHAO_MI355X_LIB=$lib timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 \
        128x28672x4096 128,1,1,3,0,0 $ld >> $O 2>> gpurun_out/$tag.err || exit $?
    done
  done
done
TORCHAO_MI355X_LIB=experiments/build/libvar_steps.so timeout -k 10 300 python -u \
  experiments/sf32_steps.py >> $O 2>> gpurun_out/$tag.err || exit $?
cat $O
