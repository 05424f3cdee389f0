#!/bin/bash
# scalar-fma int4 dequant (no v_pk_fma_f32 beside MFMAs) vs the previous build: GEMM tests, sweep
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py tests/test_gpu_gemm_tiles.py tests/test_gpu_int4.py > gpurun_out/r4_scalarfma_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_scalarfma_tests.log
[ $rc -eq 0 ] || exit $rc
for lib in old new; do
  if [ $lib = old ]; then export TORCHAO_MI355X_LIB=experiments/build/libold_pkfma.so; else unset TORCHAO_MI355X_LIB; fi
  timeout -k 10 400 python -u experiments/sweep_sf.py --paths int4 --seams 0 --shapes 128x28672x4096,128x4096x14336,128x6144x4096,128x4096x4096,64x4096x4096 --out gpurun_out/r4_sf_sweep17_$lib.jsonl > gpurun_out/r4_sf_sweep17_$lib.log 2>&1
  rc=$?; echo "sweep $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
