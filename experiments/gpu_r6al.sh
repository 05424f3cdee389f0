#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py --no-e2e > gpurun_out/bench_r6al.json 2> gpurun_out/bench_r6al.err
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r6al.json').read().strip().splitlines()[-1])
pm=d['prefill_mfma']
for k in ('int4_wo','int8_dyn'): print(k, {kk: pm[k].get(kk) for kk in ('gemm_us','attainable_us','roofline_frac','launch_floor_us','roofline_frac_with_launch_floor')})
print(d['value'], d['roofline']['frac'])"
