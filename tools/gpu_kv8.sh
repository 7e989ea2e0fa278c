#!/bin/bash
# GPU check of the widened on-load quantised forward: parity tests, then the A/B timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py -k "kv8 or dequant_pass or c3_shape" tests/test_plan_gpu.py > gpurun_out/kv8_tests.log 2>&1 || { tail -40 gpurun_out/kv8_tests.log; exit 1; }
tail -3 gpurun_out/kv8_tests.log
timeout -k 10 300 python -u tools/kv8_ab.py > gpurun_out/kv8_ab.log 2>&1 || { tail -20 gpurun_out/kv8_ab.log; exit 1; }
cat gpurun_out/kv8_ab.log
