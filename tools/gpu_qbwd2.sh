#!/bin/bash
# Quantised backwardQuery parity + A/B timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py tests/test_plan_gpu.py > gpurun_out/qbwd2_tests.log 2>&1 || { tail -40 gpurun_out/qbwd2_tests.log; exit 1; }
tail -2 gpurun_out/qbwd2_tests.log
timeout -k 10 300 python -u tools/qbwd_ab.py 2>&1 | grep -v amdgpu.ids
