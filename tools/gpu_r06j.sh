#!/bin/bash
# Round 6: block-wise on-load after making the scale loads countable: parity + A/B against the pass.
set -o pipefail
OUT=gpurun_out/r06j
mkdir -p $OUT
export TMPDIR=/tmp
#timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "blockwise or kv8" > $OUT/pytest.log 2>&1
rc=0; # $OUT/pytest.log
#[ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/kv8_ab.py "C3 fp16,C3 bf16,D64 fp16,C2c fp16" --bw 64 > $OUT/ab_bw64.txt 2>&1 || exit $?
cat $OUT/ab_bw64.txt | sed 's/on-load plan.*//'
