#!/bin/bash
# GPU-box step: the small decode GEMV shapes under one-wave-per-row-group launch shapes
# (tao_tune_int4_gemv rpw,wk,g,occ) with the shipped library and the GEMV_XPRE variant
# (experiments/variant.sh xpre=int4_gemv:-DGEMV_XPRE=1) -> gpurun_out/r5g_xpre_shapes.jsonl
cd /root/repo && export PYTHONPATH=torchao-fork_amd TMPDIR=/tmp SHAPES=4096x4096,6144x4096 && O=gpurun_out/r5g_xpre_shapes.jsonl && : > $O && for lib in "" experiments/build/libvar_xpre.so; do for t in "" 2,1,2,0 2,1,4,0 4,1,1,0 1,1,4,0 2,1,1,0; do TUNE=$t TORCHAO_MI355X_LIB=$lib timeout -k 10 120 python -u experiments/gemv_graph_time.py >> $O 2>>gpurun_out/r5g_xpre_shapes.err || exit $?; done; done; cat $O
