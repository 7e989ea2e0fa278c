#!/bin/bash
# Causal on-load quantised forward: parity, forward regressions, A/B timing, C2 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py -k "kv8 or causal" > gpurun_out/kv8c_tests.log 2>&1 || { tail -40 gpurun_out/kv8c_tests.log; exit 1; }
tail -2 gpurun_out/kv8c_tests.log
timeout -k 10 300 python -u tools/kv8_ab.py C2c,S8kc 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --no-c5 --no-mla --no-int8 > gpurun_out/kv8c_bench.json 2> gpurun_out/kv8c_bench.err || { tail -20 gpurun_out/kv8c_bench.err; exit 1; }
python -c "import json; r=json.loads(open('gpurun_out/kv8c_bench.json').read().strip().splitlines()[-1]); print('C2', r['value'], r['roofline']['kernel'])"
