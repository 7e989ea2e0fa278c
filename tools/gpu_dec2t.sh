#!/bin/bash
# Two 16-row workgroups for 17-32 rows: decode tests, then the rows-set A/B against HEAD.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_quant_gpu.py -k decode 2>&1 | tail -1 || exit 1
for i in 1 2; do
  DEC_SET=rows TAG=new timeout -k 10 200 python -u tools/dec_time.py 2>/dev/null || exit 1
  DEC_SET=rows TAG=old MFA_LIB=$PWD/tools/ablib/libmfa_old.so timeout -k 10 200 python -u tools/dec_time.py 2>/dev/null || exit 1
done
