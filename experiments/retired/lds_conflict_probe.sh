#!/bin/bash
# SQ_LDS_BANK_CONFLICT of the int4 M = 128 GEMM on each TAO_GEMM_DEBUG variant build
# (experiments/gemm_debug.sh build): which LDS traffic conflicts. usage: bash THIS OUTDIR
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for v in 0 1 2 3 4; do
  TORCHAO_MI355X_LIB="$R/experiments/build/libdbg$v.so" timeout -k 10 120 rocprofv3 -d "$OUT/v$v" -o p --output-format csv \
    --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -- python3 "$R/experiments/prof_gemm.py" int4 128 4096 4096 0 0 0 10 > "$OUT/v$v.log" 2>&1 || exit 1
done
