#!/bin/bash
# sf32 int4 kernel: rotated k order (parity + timing), step-major x debug variant, interleave
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
TORCHAO_MI355X_LIB=$B/libvar_ilrot.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > $O/r4_tests23.log 2>&1
rc=$?; echo "ilrot tests rc=$rc"; tail -1 $O/r4_tests23.log; [ $rc -eq 0 ] || exit $rc
C="128,1,1,3,0,0;128,1,1,3,0,2;128,1,2,3,0,0;128,1,4,3,0,0;64,1,4,3,0,0"
S=128x28672x4096,128x4096x4096,128x4096x14336
for lib in shipped libvar_il.so libvar_rot.so libvar_ilrot.so libvar_smaj.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; fi
  timeout -k 10 300 python -u experiments/sweep_sf.py --paths int4 --shapes $S --seams 0 --cfgs "$C" --out $O/r4_sf32_rot.jsonl > $O/r4_sf32_rot_$lib.log 2>&1
  rc=$?; echo "sweep $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
