#!/bin/bash
# Round 6, final tree: GPU suite (one process) and smoke.
set -o pipefail
OUT=gpurun_out/r06z
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
