#!/bin/bash
# Round 6: block-wise K/V on load — parity tests, then on-load vs pass A/B at C3 / D64 / C2c.
set -o pipefail
OUT=gpurun_out/r06e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py tests/test_plan_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "blockwise or kv8 or plan or golden or transposed" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/pytest.log | head -20; exit $rc; }
for bs in 64 32; do
  timeout -k 10 300 python -u tools/kv8_ab.py "C3 fp16,C3 bf16,D64 fp16,C2c fp16" --bw $bs > $OUT/ab_bw$bs.txt 2>&1 || exit $?
  cat $OUT/ab_bw$bs.txt
done
