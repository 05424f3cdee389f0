#!/bin/bash
# decode attention with the second step by LDS-DMA (tao_tune_attn 2): parity, timing, e2e A/B
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_llama_harness.py -k "attn_decode_modes" > gpurun_out/r4_attn_tests10.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -2 gpurun_out/r4_attn_tests10.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u experiments/attn_time.py --modes 0,2 --keys 128,328,512,900 > gpurun_out/r4_attn_time_lds1.jsonl 2> gpurun_out/r4_attn_time_lds1.err
rc=$?; echo "attn time rc=$rc"; cat gpurun_out/r4_attn_time_lds1.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash experiments/ab_e2e_args.sh 2 int4wo-32 "--attn_mode 0" "--attn_mode 2" > gpurun_out/r4_ab_e2e_attn_lds1.jsonl 2> gpurun_out/r4_ab_e2e_attn_lds1.err
rc=$?; echo "e2e ab rc=$rc"
python3 -c "
import json
for l in open('gpurun_out/r4_ab_e2e_attn_lds1.jsonl'):
    d=json.loads(l); print(d['args'], d['result']['decode_tokens_per_s'], d['result']['prefill_ms'])"
exit $rc
