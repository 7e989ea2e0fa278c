#!/bin/bash
# INT4 decode: parity tests, then the decode bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py -k "decode" > gpurun_out/dec4_tests.log 2>&1 || { tail -40 gpurun_out/dec4_tests.log; exit 1; }
tail -2 gpurun_out/dec4_tests.log
timeout -k 10 400 python -u bench.py --no-c5 --no-mla > gpurun_out/dec4_bench.json 2> gpurun_out/dec4_bench.err || { tail -20 gpurun_out/dec4_bench.err; exit 1; }
python - <<'PY'
import json
r = json.loads(open("gpurun_out/dec4_bench.json").read().strip().splitlines()[-1])
print(json.dumps(r.get("int8_decode"), indent=1))
PY
