#!/bin/bash
# single-fetch sweep at the Llama-3-70B prefill shapes (M = 128): int4 and int8 dyn
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u experiments/sweep_sf.py --seams 0,1 --shapes 128x10240x8192,128x8192x8192,128x57344x8192,128x8192x28672 --out gpurun_out/r4_sf_sweep_70b.jsonl > gpurun_out/r4_sf_sweep_70b.log 2>&1
rc=$?; echo "sweep rc=$rc"
exit $rc
