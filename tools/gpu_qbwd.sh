#!/bin/bash
# GPU check of the on-load quantised backwardQuery (and forward): parity tests, then the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py tests/test_plan_gpu.py > gpurun_out/qbwd_tests.log 2>&1 || { tail -60 gpurun_out/qbwd_tests.log; exit 1; }
tail -3 gpurun_out/qbwd_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/qbwd_bench.json 2> gpurun_out/qbwd_bench.err || { tail -20 gpurun_out/qbwd_bench.err; exit 1; }
python - <<'PY'
import json
r = json.loads(open("gpurun_out/qbwd_bench.json").read().strip().splitlines()[-1])
print(json.dumps(r["int8_fwd_bwd_d256"], indent=1))
print("C2", r["value"], "C5", r["fwd_bwd_d256"]["tflops"])
PY
