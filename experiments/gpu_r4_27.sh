#!/bin/bash
# 70B int4 prefill shapes on the 32x32x16 kernel: 256-column tiles (8 waves) against the routes
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
run() {  # shape cfgs
  timeout -k 10 300 python -u experiments/sweep_sf.py --paths int4 --shapes $1 --seams 0 --cfgs "$2" --out $O/r4_sf32_70b.jsonl >> $O/r4_sf32_70b.log 2>&1
}
run 128x57344x8192 "128,1,1,3,0,2;128,1,1,3,0,0;256,1,1,3,0,0;256,1,1,2,0,0;256,1,2,3,0,0" && \
run 128x10240x8192 "128,1,2,3,0,2;128,1,2,3,0,0;256,1,2,3,0,0;256,1,4,3,0,0;256,1,8,3,0,0;128,1,4,3,0,0" && \
run 128x8192x28672 "128,2,4,3,0,0;128,1,4,3,0,0;128,1,8,3,0,0;256,1,8,3,0,0;256,1,4,3,0,0;64,1,8,3,0,0" && \
run 128x8192x8192 "64,2,2,3,0,0;64,1,4,3,0,0;128,1,4,3,0,0;128,1,8,3,0,0;256,1,8,3,0,0"
rc=$?; echo "sweep rc=$rc"; exit $rc
