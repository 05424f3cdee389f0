#!/bin/bash
# decode-fused tests (incl. the 70B wqkv shape) + 70B e2e with the new fused wqkv shape
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_decode_fused.py tests/test_gpu_configs.py > gpurun_out/pytest_r6aa.log 2>&1
tail -2 gpurun_out/pytest_r6aa.log
cd torchao-fork_amd
timeout -k 10 600 python3 -u -m torchao._models.llama.generate --model_name Llama-3-70B -q int4wo-32 \
  --num_samples 3 --check_tokens 8 --write_result ../gpurun_out/e2e70b_r6aa.json > ../gpurun_out/e2e70b_r6aa.log 2>&1
tail -1 ../gpurun_out/e2e70b_r6aa.log
