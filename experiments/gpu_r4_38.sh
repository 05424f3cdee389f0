#!/bin/bash
# Final round-4 evidence: round_end.sh r4e, then the config-4 prefill kernel breakdown
cd "$(dirname "$0")/.." || exit 1
bash experiments/round_end.sh r4e || exit $?
PYTHONPATH=torchao-fork_amd timeout -k 10 300 python -u experiments/prefill_profile.py > gpurun_out/r4e_prefill_profile.jsonl 2> gpurun_out/r4e_prefill_profile.err
rc=$?; echo "prefill profile rc=$rc"; head -c 1500 gpurun_out/r4e_prefill_profile.jsonl; exit $rc
