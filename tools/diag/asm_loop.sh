#!/bin/bash
# Device asm of one HIP source + per-kernel resources + histogram of its hottest loop (development).
# Usage: tools/diag/asm_loop.sh csrc/file.hip kernel_substring [extra hipcc flags]
set -e
cd "$(dirname "$0")/../../metal-flash-attention-plus_amd"
SRC=$1; KS=$2; shift 2
OUT=/tmp/asm/$(basename $SRC .hip).s
mkdir -p /tmp/asm
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form "$@" -Icsrc \
  --cuda-device-only -S $SRC -o $OUT -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "error|remark" | \
  grep -E "error|Function Name|VGPRs:|AGPRs|Spill: [1-9]|LDS" | sed 's/.*remark: *//;s/\[-Rpass.*//' | paste - - - - || true
cd ..
python tools/diag/isa_stats.py $OUT "$KS" | head -12
L=$(python tools/diag/isa_stats.py $OUT "$KS" | awk '$1=="loop"{print $5, $2}' | sort -n | tail -1 | awk '{print $2}' | tr -d :)
echo "hottest loop $L"
python tools/diag/loop_hist.py $OUT "$KS" $L | head -${HIST:-26}
