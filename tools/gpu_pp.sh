#!/bin/bash
# pp-kernel iteration on the GPU box: its parity tests, then one-process A/B against the
# default kernels at C2 and C3 (and C4's bf16 attention).  Output: gpurun_out/TAG/
set -o pipefail
TAG=${1:-pp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_forward_pp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -15 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for cfg in C2 C3 C4A; do
  timeout -k 10 120 python -u tools/ab_fwd.py MFA_FWD_PP=0,1 --cfg $cfg --rounds 8 > "$OUT/ab_$cfg.json" 2>&1 || { echo "ab $cfg failed"; cat "$OUT/ab_$cfg.json" | tail -5; exit 1; }
  cat "$OUT/ab_$cfg.json"
done
