#!/bin/bash
# Round 6: one-process A/B of backwardQuery's next-tile DMA placement (library build).
set -o pipefail
OUT=gpurun_out/r06n
mkdir -p "$OUT"
for sh in 2,32,4096,256 4,32,4096,128 4,32,4096,64 8,32,4096,256; do
  timeout -k 10 300 python -u tools/ab_bwd.py MFA_BWDQ_DMA_AT=0,1,2 --shape $sh --rounds 6 >> "$OUT/ab.json" 2>> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 1; }
  tail -1 "$OUT/ab.json"
done
