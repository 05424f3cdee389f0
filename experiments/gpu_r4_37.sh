#!/bin/bash
# prefill attention with K and V prefetched after consumption: harness tests, timing vs the
# previous kernel (libvar_attnold), then the 8B e2e
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llama_harness.py tests/test_gpu_configs.py > $O/r4_tests37.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/r4_tests37.log; [ $rc -eq 0 ] || exit $rc
for lib in shipped libvar_attnold.so shipped libvar_attnold.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; else unset TORCHAO_MI355X_LIB; fi
  timeout -k 10 200 python -u experiments/attn_prefill_time.py --S 128,512,2048,4096 >> $O/r4_attn_prefill_pfkv.jsonl 2> $O/r4_attn_$lib.err
  rc=$?; echo "time $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
unset TORCHAO_MI355X_LIB
cd torchao-fork_amd && timeout -k 10 300 python3 -u -m torchao._models.llama.generate -q int4wo-32 --num_samples 3 > ../$O/r4_e2e_8b_pfkv.txt 2> ../$O/r4_e2e_8b_pfkv.err
rc=$?; echo "e2e rc=$rc"; tail -1 ../$O/r4_e2e_8b_pfkv.txt | cut -c1-400; exit $rc
