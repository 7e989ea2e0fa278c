#!/bin/bash
# One GPU-box pass: the GPU parity suite (one process), then the default bench line.
# Usage (from the repo root, via gpurun): bash tools/gpu_suite.sh TAG [pytest selection...]
set -o pipefail
TAG=${1:-run}; shift
SEL=${@:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
rc=$?
tail -15 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
exit $rc
