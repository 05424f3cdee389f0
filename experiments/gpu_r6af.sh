#!/bin/bash
# final library: full GPU suite, smoke, default bench line
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r6af.log 2>&1
tail -1 gpurun_out/pytest_gpu_r6af.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6af.log 2>&1
tail -1 gpurun_out/smoke_r6af.log
timeout -k 10 480 python3 -u bench.py > gpurun_out/bench_r6af.json 2> gpurun_out/bench_r6af.err
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r6af.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['e2e_decode']['decode_tokens_per_s'], d['e2e_decode']['prefill_ms'], d['unfused_w13_step']['frac'], d['config5_70b'].get('value'))"
