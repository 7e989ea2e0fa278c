#!/bin/bash
# Perf pass on the GPU box: per-config timings + rocprofv3 kernel stats (csv).
# Usage: bash tools/gpu_perf.sh TAG [perf_suite args...]
set -o pipefail
TAG=${1:-perf}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/perf_suite.py "$@" > "$OUT/perf.jsonl" 2> "$OUT/perf.err" || { echo "perf failed"; tail -20 "$OUT/perf.err"; exit 1; }
cat "$OUT/perf.jsonl"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o perf -- python3 tools/perf_suite.py --reps 4 "$@" > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>4}  {r["Name"][:110]}')
PY
