#!/bin/bash
# Round-6 first look: GPU suite, bench line, C2 stamps of the mirrored kernel and the stream kernel.
set -o pipefail
OUT=gpurun_out/r06a
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_suite.sh r06a || exit $?
timeout -k 10 120 tools/diag/fwd_stamps 16 4096 1 p 400 > $OUT/fwd_stamps_c2.txt 2>&1 || exit $?
cat $OUT/fwd_stamps_c2.txt
timeout -k 10 120 tools/diag/stream_stamps 16 4096 128 > $OUT/stream_stamps_c2.txt 2>&1 || exit $?
cat $OUT/stream_stamps_c2.txt
