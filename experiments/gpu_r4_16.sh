#!/bin/bash
# counters of the 32x32x16 int4 kernel at w1||w3 (28672 x 4096, M = 128): one / two waves per column group
cd "$(dirname "$0")/.." || exit 1
export PMC_SF_SET='run sfint4_128_28672_4096 int4 "2,128,1,1,3,0,1" 28672; run sfint4kh2_128_28672_4096 int4 "2,128,1,1,3,0,2" 28672; run sfint4bn64_128_4096_4096 int4 "2,64,2,4,2,0,0" 4096'
timeout -k 10 400 bash experiments/pmc_sf.sh gpurun_out/r4_pmc_sf32 > gpurun_out/r4_pmc_sf32.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 experiments/pmc_prefill_summary.py gpurun_out/r4_pmc_sf32 > gpurun_out/r4_pmc_sf32.jsonl
cat gpurun_out/r4_pmc_sf32.jsonl | cut -c1-1500
exit $rc
