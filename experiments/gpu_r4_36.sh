#!/bin/bash
# prefill attention: next block loaded after this block is consumed (shipped) vs at the end (libvar_pfend)
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llama_harness.py > $O/r4_tests36.log 2>&1
rc=$?; echo "harness tests rc=$rc"; tail -1 $O/r4_tests36.log; [ $rc -eq 0 ] || exit $rc
for lib in shipped libvar_pfv.so libvar_pfend.so libvar_attnold.so shipped libvar_pfv.so libvar_pfend.so libvar_attnold.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; else unset TORCHAO_MI355X_LIB; fi
  timeout -k 10 200 python -u experiments/attn_prefill_time.py --S 128,512,2048 >> $O/r4_attn_prefill_pf.jsonl 2> $O/r4_attn_$lib.err
  rc=$?; echo "time $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
