#!/bin/bash
# split-K tickets one per 128-B line (cnt_stride 32) vs packed: GEMM tests, sweep (incumbent at
# both strides, single-fetch seams at 32), stamps, e2e A/B (prefill runs the split-K GEMMs)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py tests/test_gpu_gemm_tiles.py tests/test_gpu_gemm_tile.py > gpurun_out/r4_tests6.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4_tests6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u experiments/sweep_sf.py --out gpurun_out/r4_sf_sweep6.jsonl > gpurun_out/r4_sf_sweep6.log 2>&1
rc=$?; echo "sweep rc=$rc"
[ $rc -eq 0 ] || exit $rc
TORCHAO_MI355X_LIB=experiments/build/libsfst.so timeout -k 10 240 python -u experiments/sf_stamps.py > gpurun_out/r4_sf_stamps6.log 2>&1
rc=$?; echo "stamps rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--tune cnt_stride=1" "--tune cnt_stride=32" > gpurun_out/r4_ab_e2e_cnt_stride.jsonl 2> gpurun_out/r4_ab_e2e_cnt_stride.err
rc=$?; echo "e2e ab rc=$rc"; cat gpurun_out/r4_ab_e2e_cnt_stride.jsonl | cut -c1-300
exit $rc
