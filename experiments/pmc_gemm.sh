#!/bin/bash
# Counter passes (rocprofv3 --pmc, one pass per counter group) for one GEMM configuration.
# usage: bash experiments/pmc_gemm.sh OUTDIR PATH M N K BM KG SPLITS
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -d "$OUT/p1" -o p1 --output-format csv \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  -- python3 "$R/experiments/prof_gemm.py" "$@" 20 > "$OUT/p1.log" 2>&1
timeout -k 10 120 rocprofv3 -d "$OUT/p2" -o p2 --output-format csv \
  --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC \
  -- python3 "$R/experiments/prof_gemm.py" "$@" 20 > "$OUT/p2.log" 2>&1
timeout -k 10 120 rocprofv3 -d "$OUT/p3" -o p3 --output-format csv \
  --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum \
  -- python3 "$R/experiments/prof_gemm.py" "$@" 20 > "$OUT/p3.log" 2>&1
