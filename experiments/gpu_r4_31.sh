#!/bin/bash
# Llama-3-8B e2e on one GPU, every quantization of the harness (int4wo-32, int8wo, int8dq, bf16)
cd "$(dirname "$0")/.." || exit 1
O=$PWD/gpurun_out
mkdir -p $O
cd torchao-fork_amd || exit 1
for q in int4wo-32 int8wo int8dq; do
  timeout -k 10 300 python3 -u -m torchao._models.llama.generate -q $q --num_samples 3 > $O/r4_e2e_8b_$q.txt 2> $O/r4_e2e_8b_$q.err
  rc=$?; echo "$q rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 $O/r4_e2e_8b_$q.txt >> $O/r4_e2e_8b_all.jsonl
done
