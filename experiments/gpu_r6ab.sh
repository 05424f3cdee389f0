#!/bin/bash
# int8 decode GEMV launch shapes, graph-timed
set -e
export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u experiments/sweep_int8.py --graph 4096x4096 6144x4096 14336x4096 4096x14336 28672x4096 > gpurun_out/sweep_int8_r6ab.jsonl
grep BEST gpurun_out/sweep_int8_r6ab.jsonl
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/sweep_int8_r6ab.jsonl') if l.startswith('{"path')]
for p in ('int8wo','int8dyn_fused'):
    for (N,K) in sorted({(r['N'],r['K']) for r in rows}):
        rs=[r for r in rows if r['path']==p and r['N']==N and r['K']==K]
        b=[r for r in rs if (r['rpw'],r['wk'],r['g'])==(0,0,0)]
        best=min(rs,key=lambda r:r['us'])
        print(p,N,K,'builtin',b[0]['us'] if b else None,'best',(best['rpw'],best['wk'],best['g'],best['us']))
PY
