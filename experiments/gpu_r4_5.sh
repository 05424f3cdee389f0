#!/bin/bash
# spread seam: parity, sweep (both seams), stamps; XCD-grouped decode attention: parity, timing, e2e
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > gpurun_out/r4_sf_tests5.log 2>&1
rc=$?; echo "sf tests rc=$rc"; tail -3 gpurun_out/r4_sf_tests5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llama_harness.py -k "attn_decode_modes" > gpurun_out/r4_attn_tests5.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -3 gpurun_out/r4_attn_tests5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u experiments/sweep_sf.py --out gpurun_out/r4_sf_sweep5.jsonl > gpurun_out/r4_sf_sweep5.log 2>&1
rc=$?; echo "sweep rc=$rc"
[ $rc -eq 0 ] || exit $rc
TORCHAO_MI355X_LIB=experiments/build/libsfst.so timeout -k 10 240 python -u experiments/sf_stamps.py > gpurun_out/r4_sf_stamps5.log 2>&1
rc=$?; echo "stamps rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u experiments/attn_time.py --modes 0,2 --keys 128,328,512,900 > gpurun_out/r4_attn_time_xcd.jsonl 2> gpurun_out/r4_attn_time_xcd.err
rc=$?; echo "attn time rc=$rc"; cat gpurun_out/r4_attn_time_xcd.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--attn_mode 0" "--attn_mode 2" > gpurun_out/r4_ab_e2e_attn_xcd.jsonl 2> gpurun_out/r4_ab_e2e_attn_xcd.err
rc=$?; echo "e2e ab rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash experiments/pmc_sf.sh gpurun_out/r4_pmc_sf > gpurun_out/r4_pmc_sf.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 experiments/pmc_prefill_summary.py gpurun_out/r4_pmc_sf > gpurun_out/r4_pmc_sf.jsonl
exit $rc
