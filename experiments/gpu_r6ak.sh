#!/bin/bash
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u experiments/fixed_cost_probe.py > gpurun_out/fixed_cost_r6ak.json
timeout -k 10 200 python -u experiments/fixed_cost_probe.py >> gpurun_out/fixed_cost_r6ak.json
cat gpurun_out/fixed_cost_r6ak.json
