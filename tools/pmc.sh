#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over tools/prof_kernels.py configs.
# Usage: bash tools/pmc.sh TAG config [config...]; summary -> gpurun_out/TAG/pmc_summary.txt
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for cfg in "$@"; do
  i=0; mkdir -p "$OUT/$cfg"
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/$cfg/p$i" -o run -- python3 tools/prof_kernels.py $cfg 3 > "$OUT/$cfg/p$i.log" 2>&1 || { echo "pmc pass $i $cfg failed"; tail -5 "$OUT/$cfg/p$i.log"; exit 1; }
  done
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.txt" && cat "$OUT/pmc_summary.txt"
