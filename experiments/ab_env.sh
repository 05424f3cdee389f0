#!/bin/bash
# same-box A/B of HIP runtime env knobs on the bench step
O=gpurun_out/envab.jsonl
: > $O
for r in 1 2; do
for e in "BASE=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "ROC_SYSTEM_SCOPE_SIGNAL=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
  line=$(env $e timeout -k 10 120 python bench.py --no-cpu-baseline --no-reference-gpu --no-e2e --no-extras --no-prefill --steps 50 2>/dev/null | tail -1)
  echo "{\"env\": \"$e\", \"round\": $r, \"bench\": $line}" >> $O
done
done
