#!/bin/bash
# Llama-3-70B int4wo-32 e2e with the final library (K = 8192 GEMV shapes re-tuned)
set -e
mkdir -p gpurun_out
cd torchao-fork_amd
timeout -k 10 600 python3 -u -m torchao._models.llama.generate --model_name Llama-3-70B -q int4wo-32 \
  --num_samples 3 --check_tokens 8 --write_result ../gpurun_out/e2e70b_r6x.json > ../gpurun_out/e2e70b_r6x.log 2>&1
tail -5 ../gpurun_out/e2e70b_r6x.log
