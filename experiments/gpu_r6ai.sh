#!/bin/bash
# loader-side dequantisation (tao_tune_gemm_sf_loaders 4): bit-identity tests, then timing A/B
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_gemm_sf.py -k "dequant_by_loaders or loader_waves or partials or rope" > gpurun_out/pytest_dql_r6ai.log 2>&1 || { tail -30 gpurun_out/pytest_dql_r6ai.log; exit 1; }
tail -1 gpurun_out/pytest_dql_r6ai.log
O=gpurun_out/dql_r6ai.jsonl
: > $O
for i in 1 2; do
for spec in "128x4096x4096 64,2,4,4,0,0 2" "128x4096x4096 64,2,4,3,0,0 2" "128x4096x4096 64,2,4,3,0,0 4" "128x6144x4096 64,2,2,3,0,0 2" "128x6144x4096 64,2,2,3,0,0 4" "128x4096x14336 64,2,4,4,0,0 2" "128x4096x14336 64,2,4,3,0,0 4" "128x4096x14336 64,2,4,2,0,0 4"; do
  set -- $spec
  timeout -k 10 120 python -u experiments/time_sf_cfg.py int4 $1 $2 $3 >> $O
done
done
cat $O
