#!/bin/bash
# Development: GEMM/MLA parity then one-process A/B of MFA_GEMM_IMG (C4 MLA forward, 4096^3).
set -o pipefail
OUT=gpurun_out/${1:-gimg}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_mla_gpu.py -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 180 python -u tools/ab_mla.py MFA_GEMM_IMG=0,1 --rounds 10 2>&1 | tee "$OUT/ab_mla.log" || exit 1
timeout -k 10 120 python -u tools/gemm_img_t.py 2>&1 | tee "$OUT/gemm.log"
