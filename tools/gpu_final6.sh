#!/bin/bash
# Round-6 evidence on one box: the GPU parity suite (one process), smoke, then
# tools/round_profile.sh (PMC passes, the bench line, rocprofv3 kernel stats of the same command).
set -o pipefail
TAG=${1:-r06x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -le 1 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
bash tools/round_profile.sh "$TAG" || exit $?
exit $rc
