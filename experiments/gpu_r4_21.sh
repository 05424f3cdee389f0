#!/bin/bash
# 70B routes: GEMM parity suites, then Llama-3-70B int4wo-32 e2e on one GPU
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_int4.py tests/test_gpu_int8.py tests/test_gpu_configs.py > $O/r4_tests21.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r4_tests21.log
[ $rc -eq 0 ] || exit $rc
(cd torchao-fork_amd && timeout -k 10 900 python3 -u -m torchao._models.llama.generate --model_name Llama-3-70B -q int4wo-32 --num_samples 2 --check_tokens 8 > ../$O/r4_e2e_70b.txt 2> ../$O/r4_e2e_70b.err)
rc=$?; echo "70b rc=$rc"; tail -1 $O/r4_e2e_70b.txt | cut -c1-600
exit $rc
