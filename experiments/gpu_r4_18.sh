#!/bin/bash
# where a decoded token's time goes: rocprofv3 kernel stats of the e2e harness (graph decode)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
cd torchao-fork_amd
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../gpurun_out/prof_e2e_r4 -o e2e -- python3 -m torchao._models.llama.generate -q int4wo-32 --num_samples 1 --max_new_tokens 64 --check_tokens 0 > ../gpurun_out/prof_e2e_r4.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 ../gpurun_out/prof_e2e_r4.log | cut -c1-300
f=$(find ../gpurun_out/prof_e2e_r4 -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-4 | cut -c1-200
exit $rc
