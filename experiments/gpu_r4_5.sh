#!/bin/bash
# spread seam: parity, sweep (both seams), stamps
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > gpurun_out/r4_sf_tests5.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_sf_tests5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u experiments/sweep_sf.py --out gpurun_out/r4_sf_sweep5.jsonl > gpurun_out/r4_sf_sweep5.log 2>&1
rc=$?; echo "sweep rc=$rc"
[ $rc -eq 0 ] || exit $rc
TORCHAO_MI355X_LIB=experiments/build/libsfst.so timeout -k 10 240 python -u experiments/sf_stamps.py > gpurun_out/r4_sf_stamps5.log 2>&1
rc=$?; echo "stamps rc=$rc"
exit $rc
