#!/bin/bash
# Counter passes (rocprofv3 --pmc, one group per run) for the prefill MFMA GEMMs at M = 128:
# int8-dyn and int4 at 4096x4096 and 28672x4096, auto launch shape.
# usage: bash experiments/pmc_prefill.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for cfg in "int8dyn 128 4096 4096" "int8dyn 128 28672 4096" "int4 128 4096 4096" "int4 128 28672 4096"; do
  set -- $cfg
  tag=$1_$2_$3_$4
  mkdir -p "$OUT/$tag"
  timeout -k 10 120 rocprofv3 -d "$OUT/$tag/p1" -o p1 --output-format csv \
    --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS \
    -- python3 "$R/experiments/prof_gemm.py" $1 $2 $3 $4 0 0 0 20 > "$OUT/$tag/p1.log" 2>&1
  timeout -k 10 120 rocprofv3 -d "$OUT/$tag/p2" -o p2 --output-format csv \
    --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM \
    -- python3 "$R/experiments/prof_gemm.py" $1 $2 $3 $4 0 0 0 20 > "$OUT/$tag/p2.log" 2>&1
  timeout -k 10 120 rocprofv3 -d "$OUT/$tag/p3" -o p3 --output-format csv \
    --pmc FETCH_SIZE \
    -- python3 "$R/experiments/prof_gemm.py" $1 $2 $3 $4 0 0 0 20 > "$OUT/$tag/p3.log" 2>&1
  timeout -k 10 120 rocprofv3 -d "$OUT/$tag/p4" -o p4 --output-format csv \
    --pmc GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TCP_TCC_READ_REQ_sum \
    -- python3 "$R/experiments/prof_gemm.py" $1 $2 $3 $4 0 0 0 20 > "$OUT/$tag/p4.log" 2>&1
done
echo done > "$OUT/ok"
