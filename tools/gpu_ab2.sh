#!/bin/bash
# Development: forward parity with a knob set, then one-process A/B over configs.
# Usage: bash tools/gpu_ab2.sh TAG "VAR=val" "VAR=a,b" "cfgs"
set -o pipefail
TAG=$1; KV=$2; AB=$3; CFGS=$4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
env $KV timeout -k 10 300 python -u -m pytest tests/test_forward_v2_gpu.py tests/test_forward_gpu.py \
    tests/test_golden_gpu.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for c in $CFGS; do
  timeout -k 10 180 python -u tools/ab_fwd.py "$AB" --cfg $c --rounds 10 --reps 30 2>&1 | tee -a "$OUT/ab.log" || exit 1
done
