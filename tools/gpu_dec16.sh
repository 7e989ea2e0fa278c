#!/bin/bash
# 16-row INT4 decode: decode parity tests, then the interleaved decode A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py -k "decode" > gpurun_out/dec16_tests.log 2>&1 || { tail -40 gpurun_out/dec16_tests.log; exit 1; }
tail -2 gpurun_out/dec16_tests.log
bash tools/gpu_dec4ab.sh
