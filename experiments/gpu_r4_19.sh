#!/bin/bash
# where the 32x32x16 int4 kernel's time goes: shipped vs the timing-only variants
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
O=gpurun_out/r4_sf32_debug.jsonl
: > $O
for lib in shipped 1 2 3 4; do
  if [ $lib = shipped ]; then unset TORCHAO_MI355X_LIB; else export TORCHAO_MI355X_LIB=experiments/build/libsf32dbg$lib.so; fi
  for cfg in 128,1,1,3,0,0 128,1,1,3,0,2; do
    timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 128x28672x4096 $cfg >> $O 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc lib=$lib"; exit $rc; }
  done
done
cat $O
