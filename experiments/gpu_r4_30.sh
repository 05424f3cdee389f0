#!/bin/bash
# sf32: 16-B (scale, zero) DMA pieces (shipped Z16) parity + A/B against 4-B pieces (libvar_z4)
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > $O/r4_tests30.log 2>&1
rc=$?; echo "sf tests rc=$rc"; tail -1 $O/r4_tests30.log; [ $rc -eq 0 ] || exit $rc
for lib in shipped libvar_z4.so shipped libvar_z4.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; else unset TORCHAO_MI355X_LIB; fi
  timeout -k 10 200 python -u experiments/sweep_sf.py --paths int4 --shapes 128x28672x4096 --seams 0 --cfgs "128,1,1,3,0,0;128,1,1,3,0,2;64,1,4,3,0,0" --out $O/r4_sf32_z16.jsonl >> $O/r4_sf32_z16.log 2>&1 && \
  timeout -k 10 200 python -u experiments/sweep_sf.py --paths int4 --shapes 128x57344x8192 --seams 0 --cfgs "256,1,1,3,0,0" --out $O/r4_sf32_z16.jsonl >> $O/r4_sf32_z16.log 2>&1 && \
  timeout -k 10 200 python -u experiments/sweep_sf.py --paths int4 --shapes 128x10240x8192 --seams 0 --cfgs "128,1,2,3,0,2" --out $O/r4_sf32_z16.jsonl >> $O/r4_sf32_z16.log 2>&1
  rc=$?; echo "sweep $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
