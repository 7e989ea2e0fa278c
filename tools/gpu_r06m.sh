#!/bin/bash
# Round 6: GPU suite and the bench line after moving backwardQuery's next-tile DMA after the S chain.
set -o pipefail
OUT=gpurun_out/r06m
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python - <<'PY'
import json
b = json.load(open("gpurun_out/r06m/bench.json"))
print("C2", b["value"], "C5", b["fwd_bwd_d256"], "q8", b["int8_fwd_bwd_d256"]["int8_tflops"], b["int8_fwd_bwd_d256"]["fp16_tflops"])
print("sparse bwd", b["block_sparse"]["bwd_speedup_vs_dense"], b["block_sparse"]["bwd_ms"], b["block_sparse"]["bwd_dense_ms"])
PY
