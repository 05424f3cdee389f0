#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
PYTHONPATH=torchao-fork_amd timeout -k 10 300 python -u experiments/prefill_profile.py > gpurun_out/r4_prefill_profile_fused.jsonl 2> gpurun_out/r4_prefill_profile_fused.err
rc=$?; echo "prefill profile rc=$rc"; head -c 2500 gpurun_out/r4_prefill_profile_fused.jsonl
exit $rc
