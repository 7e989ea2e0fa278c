#!/bin/bash
# decode16 occupancy A/B: (256,3) launch bounds with 512 / 768 / 1536 workgroups vs the (256,2) library.
set -o pipefail
mkdir -p gpurun_out
export MFA_DEV=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_quant_gpu.py -k "decode_int4 or decode_causal" > gpurun_out/dec16w_tests.log 2>&1 || { tail -40 gpurun_out/dec16w_tests.log; exit 1; }
tail -1 gpurun_out/dec16w_tests.log
for i in 1 2; do
  for v in old w512 w768 w1536; do
    unset MFA_LIB MFA_DECODE_WGS
    case $v in old) export MFA_LIB=$PWD/tools/ablib/libmfa_old.so;; w*) export MFA_DECODE_WGS=${v#w};; esac
    timeout -k 10 200 python -u bench.py --no-c5 --no-mla > gpurun_out/w_$v$i.json 2> gpurun_out/w_$v$i.err || { tail -20 gpurun_out/w_$v$i.err; exit 1; }
  done
done
python - <<'PY'
import json
for v in ("old", "w512", "w768", "w1536"):
    row = []
    for i in (1, 2):
        r = json.loads(open(f"gpurun_out/w_{v}{i}.json").read().strip().splitlines()[-1])["int8_decode"]
        row.append("q1 %.4f q1i4 %.4f q16 %.4f" % (r["s_q1"]["ms"], r["s_q1_int4"]["ms"], r["s_q16"]["ms"]))
    print(v, " | ".join(row))
PY
