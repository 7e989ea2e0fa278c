#!/bin/bash
# tools/dec_time.py (both shape sets) with the current library and tools/ablib/libmfa_old.so.
set -o pipefail
for set in main rows; do
  for i in 1 2; do
    DEC_SET=$set TAG=new timeout -k 10 200 python -u tools/dec_time.py 2>/dev/null || exit 1
    DEC_SET=$set TAG=old MFA_LIB=$PWD/tools/ablib/libmfa_old.so timeout -k 10 200 python -u tools/dec_time.py 2>/dev/null || exit 1
  done
done
