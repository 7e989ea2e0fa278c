#!/bin/bash
# 16-row decode at D = 256 (INT8): decode tests, then tools/dec_ab.py 2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py -k "decode" > gpurun_out/dec256_tests.log 2>&1 || { tail -40 gpurun_out/dec256_tests.log; exit 1; }
tail -1 gpurun_out/dec256_tests.log
timeout -k 10 300 python -u tools/dec_ab.py 2 > gpurun_out/dec256_ab.log 2>&1 || { tail -20 gpurun_out/dec256_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dec256_ab.log
