#!/bin/bash
# Masked on-load quantised forward: kv8 tests, then kv8_ab on the masked cases.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_quant_gpu.py -k "kv8" > gpurun_out/kv8m_tests.log 2>&1 || { tail -40 gpurun_out/kv8m_tests.log; exit 1; }
tail -1 gpurun_out/kv8m_tests.log
timeout -k 10 400 python -u tools/kv8_ab.py C2c,S8kc,D64c,C5c,B4c,S8kw,C5w > gpurun_out/kv8m_ab.log 2>&1 || { tail -20 gpurun_out/kv8m_ab.log; exit 1; }
sed -e 's/on-load plan.*//' gpurun_out/kv8m_ab.log
