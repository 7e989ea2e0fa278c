#!/bin/bash
# Round evidence on the GPU box: bench.py line, rocprofv3 kernel stats of the same command,
# HBM traffic PMC passes of the headline kernels.  Output: gpurun_out/TAG/
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/pmc.sh "$TAG/pmc" c2 c3 c3i8 c5f c5q c5kv dec4 dec8 > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; tail -20 "$OUT/pmc.log"; exit 1; }
python3 tools/pmc_traffic.py "$OUT/pmc" > "$OUT/pmc_traffic.json"
# bench.py reads the newest profiles/r*_pmc_traffic.json for roofline.traffic: this round's.
cp "$OUT/pmc_traffic.json" "profiles/${TAG}_pmc_traffic.json"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 bench.py --no-cpu > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>4}  {r["Name"][:100]}')
PY
