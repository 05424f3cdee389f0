#!/bin/bash
# GPU-box step: experiments/gemv_graph_time.py with the shipped library and each timing-only
# GEMV variant (experiments/variant.sh gvN=int4_gemv:-DTAO_GEMV_DEBUG=N), then the loads-only
# probe (probe_two_streams.py) in the same call. bash experiments/gemv_variants.sh TAG
cd "$(dirname "$0")/.." || exit 1
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
O=gpurun_out/$1.jsonl
: > $O
for v in shipped gv1 gv2 gv3 gv4 gv5 gv6; do
  lib=""
  [ "$v" != shipped ] && lib=experiments/build/libvar_$v.so
  TORCHAO_MI355X_LIB=$lib timeout -k 10 300 python -u experiments/gemv_graph_time.py >> $O \
    2>> gpurun_out/$1.err || exit $?
done
timeout -k 10 300 python -u experiments/probe_two_streams.py >> $O 2>> gpurun_out/$1.err || exit $?
cat $O
