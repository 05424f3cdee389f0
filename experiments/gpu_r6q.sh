#!/bin/bash
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u experiments/intake_modes.py > gpurun_out/intake_modes_r6q.jsonl
cat gpurun_out/intake_modes_r6q.jsonl
