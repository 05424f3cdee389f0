#!/bin/bash
# sf32 int4 kernel: DMA-interleave variant parity + sweep against the shipped build, BN 256 shapes
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
IL=$PWD/experiments/build/libvar_il.so
# (the IL build passed tests/test_gpu_gemm_sf.py: profiles/r4_pytest_gemm_sf_il.log)
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llama_harness.py -k add_rmsnorm > $O/r4_tests22.log 2>&1
rc=$?; echo "add_rmsnorm test rc=$rc"; tail -1 $O/r4_tests22.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -u experiments/time_addnorm.py > $O/r4_time_addnorm.jsonl && \
TORCHAO_MI355X_LIB=$PWD/experiments/build/libvar_addloop.so timeout -k 10 100 python -u experiments/time_addnorm.py >> $O/r4_time_addnorm.jsonl
rc=$?; echo "addnorm timing rc=$rc"; cat $O/r4_time_addnorm.jsonl; [ $rc -eq 0 ] || exit $rc

C="128,1,1,3,0,0;128,1,1,3,0,2;128,1,2,3,0,0;256,1,1,3,0,0;256,1,2,3,0,0;256,1,1,2,0,0;128,1,4,3,0,0;256,1,4,3,0,0;128,1,8,3,0,0;256,1,8,3,0,0;64,1,4,3,0,0;64,1,8,3,0,0"
S=128x28672x4096,128x4096x4096,128x6144x4096,128x4096x14336
for lib in shipped il; do
  if [ $lib = il ]; then export TORCHAO_MI355X_LIB=$IL; fi
  timeout -k 10 400 python -u experiments/sweep_sf.py --paths int4 --shapes $S --seams 0 --cfgs "$C" --out $O/r4_sf32_il.jsonl > $O/r4_sf32_il_$lib.log 2>&1
  rc=$?; echo "sweep $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
