#!/bin/bash
# intake probe test + sf tests, wqkv GEMV launch-shape A/B, bench line with the intake block
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_sf.py > gpurun_out/pytest_sf_r6p.log 2>&1
timeout -k 10 200 python -u experiments/ab_gemv_shape.py 6144x4096 "2,2,4,0;2,1,4,0;2,1,1,0" 6 > gpurun_out/ab_wqkv_shape_r6p.jsonl
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-e2e > gpurun_out/bench_r6p.json 2> gpurun_out/bench_r6p.err
tail -2 gpurun_out/pytest_sf_r6p.log; cat gpurun_out/ab_wqkv_shape_r6p.jsonl
python - <<'PY'
import json
d=json.loads(open('gpurun_out/bench_r6p.json').read().strip().splitlines()[-1])
pm=d.get('prefill_mfma',{})
for k in ('int4_wo','int8_dyn'):
    v=pm.get(k,{}); print(k, {kk: v.get(kk) for kk in ('gemm_us','graph_us','roofline_frac','intake_probe','intake_probe_sf_int8')})
print('value', d['value'], d['ms_per_step'], d['roofline']['frac'])
PY
