#!/bin/bash
# per-token kernel budget of the e2e decode (config 4) on the final library
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
cd torchao-fork_amd
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ../gpurun_out/e2e_prof_r6v -o e2e -- \
  python3 -m torchao._models.llama.generate -q int4wo-32 --num_samples 1 --max_new_tokens 96 --check_tokens 0 > ../gpurun_out/e2e_prof_r6v.log 2>&1
cd ..
python3 experiments/e2e_summary.py "$(find gpurun_out/e2e_prof_r6v -name "*kernel_trace.csv" | head -1)" 96 > gpurun_out/e2e_budget_r6v.txt
cat gpurun_out/e2e_budget_r6v.txt | head -40
