#!/bin/bash
# Round 6: stream-kernel stamps at C2, the phase-2 DMA ablation of the mirrored kernel, INT8 A/B.
set -o pipefail
OUT=gpurun_out/r06c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/ab_fwd.py MFA_I8_BIAS=0,1 --cfg C3I8 --rounds 10 > $OUT/ab_i8_bias.json 2>&1 || exit $?
cat $OUT/ab_i8_bias.json
timeout -k 10 120 tools/diag/stream_stamps 16 4096 128 > $OUT/stream_stamps_c2.txt 2>&1 || exit $?
cat $OUT/stream_stamps_c2.txt
timeout -k 10 120 tools/diag/fwd_stamps_p2 16 4096 1 p 400 > $OUT/fwd_stamps_p2_c2.txt 2>&1 || exit $?
cat $OUT/fwd_stamps_p2_c2.txt
