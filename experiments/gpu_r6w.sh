#!/bin/bash
# launch-shape sweep of the decode-fused GEMVs (RMSNorm prologue + SwiGLU / RoPE) after the
# byte-permute decode
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u experiments/bench_decode.py --sweep --model ${MODEL:-8b} > gpurun_out/bench_decode_sweep_${TAG:-r6w}.jsonl
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/bench_decode_sweep_' + __import__("os").environ.get("TAG","r6w") + '.jsonl')]
for op in sorted({r['op'] for r in rows}):
    rs=[r for r in rows if r['op']==op]
    base=[r for r in rs if tuple(r['tune'])==(0,0,0,0)][0]
    best=sorted(rs,key=lambda r:r['fused_us'])[:4]
    print(op,'builtin',base['fused_us'],'gemv_only',base.get('gemv_only_us'),'best',[(r['tune'],r['fused_us']) for r in best])
PY
