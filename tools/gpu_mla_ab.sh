#!/bin/bash
# Absorbed-MLA decode A/B: current library vs tools/ablib/libmfa_old.so, interleaved.
set -o pipefail
for i in 1 2 3; do
  TAG=new timeout -k 10 120 python -u tools/mla_dec_time.py 2>/dev/null || exit 1
  TAG=old MFA_LIB=$PWD/tools/ablib/libmfa_old.so timeout -k 10 120 python -u tools/mla_dec_time.py 2>/dev/null || exit 1
done
