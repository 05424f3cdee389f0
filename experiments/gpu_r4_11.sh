#!/bin/bash
# prefill attention vs SDPA at long prompts; where the config-4 prefill spends its time now
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u experiments/attn_prefill_time.py > gpurun_out/r4_attn_prefill_time.jsonl 2> gpurun_out/r4_attn_prefill_time.err
rc=$?; echo "attn prefill rc=$rc"; cat gpurun_out/r4_attn_prefill_time.jsonl
[ $rc -eq 0 ] || exit $rc
PYTHONPATH=torchao-fork_amd timeout -k 10 300 python -u experiments/prefill_profile.py > gpurun_out/r4_prefill_profile.jsonl 2> gpurun_out/r4_prefill_profile.err
rc=$?; echo "prefill profile rc=$rc"; head -c 3000 gpurun_out/r4_prefill_profile.jsonl
exit $rc
