#!/bin/bash
# SwiGLU and RoPE + KV epilogues: parity, e2e prefill A/B
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py -k "swiglu or rope" > gpurun_out/r4_epi_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4_epi_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--prefill_swiglu 0 --prefill_rope 0" "--prefill_swiglu 1 --prefill_rope 0" "--prefill_swiglu 1 --prefill_rope 1" > gpurun_out/r4_ab_e2e_epi.jsonl 2> gpurun_out/r4_ab_e2e_epi.err
rc=$?; echo "e2e ab rc=$rc"
python3 -c "
import json
for l in open('gpurun_out/r4_ab_e2e_epi.jsonl'):
    d=json.loads(l); r=d['result']; print(d['args'], r['decode_tokens_per_s'], r['prefill_ms'], r.get('graph_eager_token_match'))"
exit $rc
