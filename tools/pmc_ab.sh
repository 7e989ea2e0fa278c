#!/bin/bash
# PMC passes (P1 issue/wait, P2 LDS/SALU) of one prof_kernels config under two env settings.
# Usage: bash tools/pmc_ab.sh TAG cfg "ENV=a" "ENV=b"
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
for E in "$@"; do
  d="$OUT/${E//=/_}"; mkdir -p "$d"; i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    env $E true
    export ${E%%=*}=${E#*=}
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$d/p$i" -o run -- python3 tools/prof_kernels.py $CFG 3 > "$d/p$i.log" 2>&1 || { echo "pmc pass $i $E failed"; tail -5 "$d/p$i.log"; exit 1; }
  done
  echo "#### $E"; python3 tools/pmc_summary.py "$d"
done
