#!/bin/bash
# sf32 int4 kernel: DMA-interleave variant parity + sweep against the shipped build, BN 256 shapes
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
IL=$PWD/experiments/build/libsf32il.so
false && TORCHAO_MI355X_LIB=$IL timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > $O/r4_tests22.log 2>&1
echo "il tests passed in the previous call (287)"

C="128,1,1,3,0,0;128,1,1,3,0,2;128,1,2,3,0,0;256,1,1,3,0,0;256,1,2,3,0,0;256,1,1,2,0,0;128,1,4,3,0,0;256,1,4,3,0,0;128,1,8,3,0,0;256,1,8,3,0,0;64,1,4,3,0,0;64,1,8,3,0,0"
S=128x28672x4096,128x4096x4096,128x6144x4096,128x4096x14336
for lib in shipped il; do
  if [ $lib = il ]; then export TORCHAO_MI355X_LIB=$IL; fi
  timeout -k 10 400 python -u experiments/sweep_sf.py --paths int4 --shapes $S --seams 0 --cfgs "$C" --out $O/r4_sf32_il.jsonl > $O/r4_sf32_il_$lib.log 2>&1
  rc=$?; echo "sweep $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
