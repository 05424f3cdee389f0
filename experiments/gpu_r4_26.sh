#!/bin/bash
# prefill attention: K/V register double buffer (shipped) vs the previous kernel (libvar_attnold)
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out
mkdir -p $O
B=$PWD/experiments/build
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llama_harness.py > $O/r4_tests26.log 2>&1
rc=$?; echo "harness tests rc=$rc"; tail -1 $O/r4_tests26.log; [ $rc -eq 0 ] || exit $rc
for lib in shipped libvar_attnold.so shipped libvar_attnold.so; do
  if [ $lib != shipped ]; then export TORCHAO_MI355X_LIB=$B/$lib; else unset TORCHAO_MI355X_LIB; fi
  timeout -k 10 200 python -u experiments/attn_prefill_time.py --S 128,512,2048 >> $O/r4_attn_prefill_db.jsonl 2> $O/r4_attn_$lib.err
  rc=$?; echo "time $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
