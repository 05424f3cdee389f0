#!/bin/bash
# MFMA utilisation evidence for the prefill GEMMs (rocprofv3 kernel trace + one --pmc pass per
# config), summarised by experiments/mfma_summary.py.
# usage: bash experiments/pmc_mfma.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for cfg in "int8dyn 128 4096 4096" "int4 128 4096 4096" "int8dyn 128 14336 4096" "int8dyn 512 14336 4096"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/$tag/kt" -o kt --output-format csv \
    -- python3 "$R/experiments/prof_gemm.py" $cfg 0 0 0 30 > "$OUT/$tag.kt.log" 2>&1
  timeout -s KILL 90 rocprofv3 -d "$OUT/$tag/pmc" -o pmc --output-format csv \
    --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -- python3 "$R/experiments/prof_gemm.py" $cfg 0 0 0 30 > "$OUT/$tag.pmc.log" 2>&1
done
