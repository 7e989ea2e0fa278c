#!/bin/bash
# Round 6: C2 light-pair prologue delay A/B (one process per split, interleaved delays).
set -o pipefail
OUT=gpurun_out/r06d
mkdir -p $OUT
export TMPDIR=/tmp
for sp in 8 12 4; do
  MFA_FWD_DELAY_SPLIT=$sp timeout -k 10 200 python -u tools/ab_fwd.py MFA_FWD_DELAY=0,4,8,12 --cfg C2 --rounds 12 > $OUT/ab_delay_s$sp.json 2>&1 || exit $?
  echo "split $sp: $(cat $OUT/ab_delay_s$sp.json)"
done
