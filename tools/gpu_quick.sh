#!/bin/bash
# Quick GPU iteration: selected GPU tests, then a reduced bench line.
# Usage: bash tools/gpu_quick.sh TAG "pytest selection" "bench flags"
set -o pipefail
TAG=$1; SEL=$2; BFLAGS=$3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?
  tail -25 "$OUT/pytest.log"
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
if [ -n "$BFLAGS" ]; then
  timeout -k 10 400 python -u bench.py $BFLAGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
fi
