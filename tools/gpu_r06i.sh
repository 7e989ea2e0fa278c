#!/bin/bash
set -o pipefail
OUT=gpurun_out/r06i
mkdir -p $OUT
timeout -k 10 120 tools/diag/bwd_stamps 1 16 4096 128 8 > $OUT/bwd_stamps_band8.txt 2>&1 || exit $?
cat $OUT/bwd_stamps_band8.txt
