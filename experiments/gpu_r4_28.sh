#!/bin/bash
# sf32 bn 256 tests; 70B 57344x8192 int4 launch shapes with and without the DMA interleave
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > $O/r4_tests28.log 2>&1
rc=$?; echo "sf tests rc=$rc"; tail -1 $O/r4_tests28.log; [ $rc -eq 0 ] || exit $rc
C="128,1,1,3,0,2;128,1,1,3,0,0;256,1,1,3,0,0;256,1,1,2,0,0"
for lib in shipped libvar_il0.so shipped libvar_il0.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; else unset TORCHAO_MI355X_LIB; fi
  timeout -k 10 300 python -u experiments/sweep_sf.py --paths int4 --shapes 128x57344x8192,128x28672x4096 --seams 0 --cfgs "$C" --out $O/r4_sf32_70b_il.jsonl >> $O/r4_sf32_70b_il.log 2>&1
  rc=$?; echo "sweep $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
