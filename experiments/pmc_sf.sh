#!/bin/bash
# Counter passes (rocprofv3 --pmc, one group per run) of the routed prefill GEMMs at M = 128,
# 4096x4096, int8 dyn and int4: the incumbent and single-fetch launch shapes given as
# "tag path sfcfg" triples (sfcfg "-" = incumbent). usage: bash experiments/pmc_sf.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
run() {  # tag path sfcfg [N]
  local tag=$1 path=$2 sf=$3 n=${4:-4096}
  mkdir -p "$OUT/$tag"
  local envs=""
  [ "$sf" != "-" ] && envs="PROF_SF=$sf"
  for pass in 1 2 3 4; do
    case $pass in
      1) pmc="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS" ;;
      2) pmc="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM" ;;
      3) pmc="FETCH_SIZE" ;;
      4) pmc="GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TCP_TCC_READ_REQ_sum" ;;
    esac
    env $envs timeout -k 10 120 rocprofv3 -d "$OUT/$tag/p$pass" -o p$pass --output-format csv \
      --pmc $pmc -- python3 "$R/experiments/prof_gemm.py" $path 128 $n 4096 0 0 0 20 \
      > "$OUT/$tag/p$pass.log" 2>&1
  done
}
if [ -n "$PMC_SF_SET" ]; then
  eval "$PMC_SF_SET"
else
  run int8dyn_128_4096_4096 int8dyn -
  run int4_128_4096_4096 int4 -
  run sfint8_128_4096_4096 int8dyn "2,64,4,4,3,0,128"
  run sfint4_128_4096_4096 int4 "2,64,2,4,2,0,0"
fi
echo done > "$OUT/ok"
