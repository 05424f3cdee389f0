#!/bin/bash
# round 4: single-fetch GEMM parity tests, then a sweep against the incumbent
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_gemm_sf.py > gpurun_out/r4_sf_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/r4_sf_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u experiments/sweep_sf.py --out gpurun_out/r4_sf_sweep1.jsonl > gpurun_out/r4_sf_sweep1.log 2>&1
rc=$?
echo "sweep rc=$rc"
tail -3 gpurun_out/r4_sf_sweep1.log
exit $rc
