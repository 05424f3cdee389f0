#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py -k "register or deterministic or graph" > gpurun_out/r4_sf_tests3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_sf_tests3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u experiments/sweep_sf.py --reg 1 --out gpurun_out/r4_sf_sweep3.jsonl > gpurun_out/r4_sf_sweep3.log 2>&1
rc=$?; echo "sweep rc=$rc"
[ $rc -eq 0 ] || exit $rc
TORCHAO_MI355X_LIB=experiments/build/libsfst.so timeout -k 10 240 python -u experiments/sf_stamps.py > gpurun_out/r4_sf_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; tail -3 gpurun_out/r4_sf_stamps.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u experiments/ref_prefill.py > gpurun_out/r4_ref_prefill.log 2>&1
rc=$?; echo "ref rc=$rc"; tail -2 gpurun_out/r4_ref_prefill.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u experiments/ab_fenced.py > gpurun_out/r4_ab_fenced.log 2>&1
rc=$?; echo "fenced rc=$rc"; tail -2 gpurun_out/r4_ab_fenced.log
exit $rc
