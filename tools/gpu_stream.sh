#!/bin/bash
# Stream-split causal forward: parity tests, stamps, one-process A/B against the mirrored kernel.
set -o pipefail
OUT=gpurun_out/${1:-stream}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_forward_stream_gpu.py "tests/test_quant_gpu.py::test_transposed_quantized_kv_matches_row_major" -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/diag/stream_stamps 16 4096 128 > "$OUT/stamps.txt" 2>&1 || { tail -20 "$OUT/stamps.txt"; exit 1; }
cat "$OUT/stamps.txt"
timeout -k 10 200 python -u tools/ab_fwd.py MFA_FWD_STREAM=0,1 --cfg C2 --rounds 8 > "$OUT/ab_c2.txt" 2>&1 || { tail -20 "$OUT/ab_c2.txt"; exit 1; }
cat "$OUT/ab_c2.txt"
