#!/bin/bash
# Development: forward parity suite with a dispatch knob set, then one-process A/B.
# Usage: bash tools/gpu_chain.sh TAG KNOBVAR=val "a,b" "cfgs"
set -o pipefail
TAG=${1:-chain}; KV=${2:-MFA_FWD_PAIR=c}; AB=${3:-MFA_FWD_PAIR=o,c}; CFGS=${4:-"C2 C2D64"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
env $KV timeout -k 10 300 python -u -m pytest tests/test_forward_v2_gpu.py tests/test_forward_gpu.py \
    tests/test_golden_gpu.py tests/test_plan_gpu.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for c in $CFGS; do
  timeout -k 10 180 python -u tools/ab_fwd.py "$AB" --cfg $c --rounds 10 --reps 40 2>&1 | tee -a "$OUT/ab.log" || exit 1
done
