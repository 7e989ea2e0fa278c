#!/bin/bash
# Development: quantised-forward parity with a knob set, then one-process A/B at C3 INT8.
# Usage: bash tools/gpu_i8.sh TAG KNOBVAR=val "VAR=a,b"
set -o pipefail
TAG=${1:-i8}; KV=${2:-MFA_I8_BK=p}; AB=${3:-MFA_I8_BK=1,p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
env $KV timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py tests/test_plan_gpu.py -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 180 python -u tools/ab_fwd.py "$AB" --cfg C3I8 --rounds 10 --reps 20 2>&1 | tee -a "$OUT/ab.log"
