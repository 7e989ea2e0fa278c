#!/bin/bash
# GPU box: full -m gpu suite, then interleaved A/B of forward variants (development).
# Usage: bash tools/gpu_ab.sh TAG "KNOB=a,b" "cfg1 cfg2 ..."
set -o pipefail
TAG=${1:-ab}; KNOB=${2:-MFA_FWD_SHARE=0,1}; CFGS=${3:-"C2 C3"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
${PYTEST_ENV:-} timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for c in $CFGS; do
  timeout -k 10 180 python -u tools/ab_fwd.py "$KNOB" --cfg $c --rounds 10 --reps 40 2>&1 | tee -a "$OUT/ab.log" || exit 1
done
