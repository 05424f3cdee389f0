#!/bin/bash
# Prefill GEMM counter passes (routed kernels, final code) -> r4d_pmc_prefill
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
timeout -k 10 600 bash experiments/pmc_prefill.sh gpurun_out/r4d_pmc_prefill > $O/r4d_pmc_prefill.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 experiments/pmc_prefill_summary.py gpurun_out/r4d_pmc_prefill > $O/r4d_pmc_prefill.jsonl
exit $rc
