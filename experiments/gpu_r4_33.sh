#!/bin/bash
# 16x16 int4 single-fetch kernel at 8B's wqkv / wo / w2: 3-4 stages with the DMA interleave
# (libvar_sfil) against the shipped build's 2-stage routes
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
C="64,2,4,2,0;64,2,4,3,0;64,2,4,4,0;64,2,2,3,0;64,2,2,4,0"
for lib in shipped libvar_sfil.so shipped libvar_sfil.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; else unset TORCHAO_MI355X_LIB; fi
  timeout -k 10 300 python -u experiments/sweep_sf.py --paths int4 --shapes 128x4096x4096,128x6144x4096,128x4096x14336 --seams 0,1 --cfgs "$C" --out $O/r4_sf_il_ns.jsonl >> $O/r4_sf_il_ns.log 2>&1
  rc=$?; echo "sweep $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
