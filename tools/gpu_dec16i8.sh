#!/bin/bash
# 16-row decode for INT8 too: decode tests, then default vs MFA_DECODE16=4 (INT8 on the 32-row
# kernel), interleaved, same library.
set -o pipefail
mkdir -p gpurun_out
export MFA_DEV=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py -k "decode" > gpurun_out/dec16i8_tests.log 2>&1 || { tail -40 gpurun_out/dec16i8_tests.log; exit 1; }
tail -1 gpurun_out/dec16i8_tests.log
for i in 1 2 3; do
  for v in d16 d32; do
    unset MFA_DECODE16
    [ $v = d32 ] && export MFA_DECODE16=4
    timeout -k 10 200 python -u bench.py --no-c5 --no-mla > gpurun_out/x_$v$i.json 2> gpurun_out/x_$v$i.err || { tail -20 gpurun_out/x_$v$i.err; exit 1; }
  done
done
python - <<'PY'
import json
for v in ("d16", "d32"):
    row = []
    for i in (1, 2, 3):
        r = json.loads(open(f"gpurun_out/x_{v}{i}.json").read().strip().splitlines()[-1])["int8_decode"]
        row.append("q1 %.4f q1i4 %.4f q16 %.4f" % (r["s_q1"]["ms"], r["s_q1_int4"]["ms"], r["s_q16"]["ms"]))
    print(v, " | ".join(row))
PY
