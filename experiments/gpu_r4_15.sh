#!/bin/bash
# 32x32x16 int4 kernel with k halves (8 waves): parity, sweep of the int4 prefill shapes
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py -k "k_halves or sf_int4 or swiglu" > gpurun_out/r4_kh_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_kh_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u experiments/sweep_sf.py --paths int4 --seams 0 --shapes 128x28672x4096,128x4096x14336,128x6144x4096,128x4096x4096 --out gpurun_out/r4_sf_sweep15.jsonl > gpurun_out/r4_sf_sweep15.log 2>&1
rc=$?; echo "sweep rc=$rc"
exit $rc
