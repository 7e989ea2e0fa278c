#!/bin/bash
# Round 6: backwardQuery next-tile DMA placement (top / after S chain / after dP chain), stamped
# builds alternated twice per shape.
set -o pipefail
OUT=gpurun_out/r06l
mkdir -p "$OUT"
for rep in 1 2; do
  for args in "1 16 4096 128 0 1" "2 32 4096 256 0 1" "1 16 4096 128 8 1"; do
    for v in bwd_stamps bwd_stamps_qdma1 bwd_stamps_qdma2; do
      echo "== $v $args (rep $rep)" >> "$OUT/all.txt"
      timeout -k 10 60 tools/diag/$v $args >> "$OUT/all.txt" 2>&1 || exit 1
    done
  done
done
grep -E "^==|^bwd_q|S chain|dP chain|dQ chain|DMA issue|barrier" "$OUT/all.txt"
