#!/bin/bash
# Process-level A/B of the decode lines: current library vs tools/ablib/libmfa_old.so,
# interleaved three times.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export MFA_LIB=$PWD/tools/ablib/libmfa_old.so; else unset MFA_LIB; fi
    timeout -k 10 200 python -u bench.py --no-c5 --no-mla > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || { tail -20 gpurun_out/ab_$v$i.err; exit 1; }
  done
done
python - <<'PY'
import json
for v in ("new", "old"):
    row = []
    for i in (1, 2, 3):
        r = json.loads(open(f"gpurun_out/ab_{v}{i}.json").read().strip().splitlines()[-1])["int8_decode"]
        row.append("q1 %.4f q1i4 %.4f q16 %.4f" % (r["s_q1"]["ms"], r["s_q1_int4"]["ms"], r["s_q16"]["ms"]))
    print(v, " | ".join(row))
PY
