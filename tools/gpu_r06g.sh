#!/bin/bash
# Round 6: where the masked key phase's prologue goes (block-sparse band 8 of 32, B1 H16 S4096 D128).
set -o pipefail
OUT=gpurun_out/r06g
mkdir -p $OUT
timeout -k 10 120 tools/diag/bwd_stamps 1 16 4096 128 8 > $OUT/bwd_stamps_band8.txt 2>&1 || exit $?
cat $OUT/bwd_stamps_band8.txt
timeout -k 10 120 tools/diag/bwd_stamps 1 16 4096 128 0 > $OUT/bwd_stamps_dense.txt 2>&1 || exit $?
cat $OUT/bwd_stamps_dense.txt
