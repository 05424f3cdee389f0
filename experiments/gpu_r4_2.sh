#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
TORCHAO_MI355X_LIB=experiments/build/libsfst.so timeout -k 10 240 python -u experiments/sf_stamps.py > gpurun_out/r4_sf_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; tail -12 gpurun_out/r4_sf_stamps.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u experiments/ref_prefill.py > gpurun_out/r4_ref_prefill.log 2>&1
rc=$?; echo "ref rc=$rc"; tail -3 gpurun_out/r4_ref_prefill.log
exit $rc
