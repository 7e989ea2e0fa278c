#!/bin/bash
# Decode split partials A/B: decode tests, then tools/dec_time.py (both shape sets) with the
# current library and tools/ablib/libmfa_old.so, interleaved.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_quant_gpu.py -k decode 2>&1 | tail -1 || exit 1
for set in main rows; do
  for i in 1 2; do
    DEC_SET=$set TAG=new timeout -k 10 200 python -u tools/dec_time.py 2>/dev/null || exit 1
    DEC_SET=$set TAG=old MFA_LIB=$PWD/tools/ablib/libmfa_old.so timeout -k 10 200 python -u tools/dec_time.py 2>/dev/null || exit 1
  done
done
