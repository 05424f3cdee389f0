#!/bin/bash
# sf32 int4 kernel: per-instruction vs per-byte cost of the LDS-DMA pieces (timing-only variants)
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
C="128,1,1,3,0,0;64,1,4,3,0,0"
S=128x28672x4096,128x4096x4096
for lib in shipped libvar_il0.so libvar_noz.so libvar_now.so libvar_nodma.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; fi
  timeout -k 10 300 python -u experiments/sweep_sf.py --paths int4 --shapes $S --seams 0 --cfgs "$C" --out $O/r4_sf32_dmacost.jsonl > $O/r4_sf32_dmacost_$lib.log 2>&1
  rc=$?; echo "sweep $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
