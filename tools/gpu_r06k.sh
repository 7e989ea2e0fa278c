#!/bin/bash
# Round 6: backwardQuery phase stamps (dense and band-8 sparse at D = 128, dense D = 256) and the
# key phase dense at D = 128 beside the band-8 run already in profiles/.
set -o pipefail
OUT=gpurun_out/r06k
mkdir -p "$OUT"
B=tools/diag/bwd_stamps
timeout -k 10 60 $B 1 16 4096 128 0 1 > "$OUT/q_d128_dense.txt" 2>&1 && cat "$OUT/q_d128_dense.txt" &&
timeout -k 10 60 $B 1 16 4096 128 8 1 > "$OUT/q_d128_band8.txt" 2>&1 && cat "$OUT/q_d128_band8.txt" &&
timeout -k 10 60 $B 1 16 4096 128 32 1 > "$OUT/q_d128_band32.txt" 2>&1 && cat "$OUT/q_d128_band32.txt" &&
timeout -k 10 60 $B 2 32 4096 256 0 1 > "$OUT/q_d256_dense.txt" 2>&1 && cat "$OUT/q_d256_dense.txt" &&
timeout -k 10 60 $B 1 16 4096 128 0 0 > "$OUT/kv_d128_dense.txt" 2>&1 && cat "$OUT/kv_d128_dense.txt" &&
timeout -k 10 60 $B 1 16 4096 128 32 0 > "$OUT/kv_d128_band32.txt" 2>&1 && cat "$OUT/kv_d128_band32.txt" &&
timeout -k 10 60 $B 1 16 4096 128 8 0 > "$OUT/kv_d128_band8.txt" 2>&1 && cat "$OUT/kv_d128_band8.txt"
