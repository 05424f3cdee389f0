#!/bin/bash
# 32x32x16 int4 kernel with 64-row tiles: parity, then launch shapes against the routes
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > $O/r4_tests34.log 2>&1
rc=$?; echo "sf tests rc=$rc"; tail -1 $O/r4_tests34.log; [ $rc -eq 0 ] || exit $rc
run() {
  timeout -k 10 300 python -u experiments/sweep_sf.py --paths int4 --shapes $1 --seams 0 --cfgs "$2" --out $O/r4_sf32_bm64.jsonl >> $O/r4_sf32_bm64.log 2>&1
}
for pass in 1 2; do
run 128x28672x4096 "128,1,1,3,0,0;256,1,1,3,0,64;256,1,1,4,0,64;256,1,1,2,0,64;128,1,1,3,0,64;128,1,1,4,0,64" && \
run 128x57344x8192 "256,1,1,3,0,0;256,1,1,3,0,64;256,1,1,4,0,64" && \
run 128x10240x8192 "128,1,2,3,0,2;256,1,2,3,0,64;128,1,2,3,0,64;256,1,4,3,0,64" && \
run 128x4096x14336 "256,1,4,3,0,64;128,1,4,3,0,64;128,1,2,4,0,64" && \
run 128x6144x4096 "256,1,4,3,0,64;128,1,2,3,0,64;128,1,4,3,0,64"
rc=$?; echo "sweep pass $pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
