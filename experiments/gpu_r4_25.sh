#!/bin/bash
# gemm_sf: DMA-interleave variant (TAO_SF_IL=1) parity + routed-shape timing against the shipped build
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
TORCHAO_MI355X_LIB=$B/libvar_sfil.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > $O/r4_tests25.log 2>&1
rc=$?; echo "sfil tests rc=$rc"; tail -1 $O/r4_tests25.log; [ $rc -eq 0 ] || exit $rc
for lib in shipped libvar_sfil.so shipped libvar_sfil.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; else unset TORCHAO_MI355X_LIB; fi
  timeout -k 10 300 python -u experiments/time_routes.py --big >> $O/r4_routes_sfil.jsonl 2> $O/r4_routes_$lib.err
  rc=$?; echo "routes $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
