#!/bin/bash
# Llama-3-70B int4wo-32 e2e on one GPU with the 256-column w1||w3 route
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
(cd torchao-fork_amd && timeout -k 10 900 python3 -u -m torchao._models.llama.generate --model_name Llama-3-70B -q int4wo-32 --num_samples 2 --check_tokens 8 > ../$O/r4_e2e_70b_b.txt 2> ../$O/r4_e2e_70b_b.err)
rc=$?; echo "70b rc=$rc"; tail -1 $O/r4_e2e_70b_b.txt | cut -c1-700
exit $rc
