#!/bin/bash
# One GPU-box pass: parity tests, headline bench, rocprofv3 kernel stats of the bench.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench -- python3 bench.py --no-cpu \
    > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cut -c1-200 {}
