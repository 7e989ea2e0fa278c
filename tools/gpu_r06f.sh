#!/bin/bash
# Round 6: block-wise on-load parity + A/B (fma_mix fast path), on-load INT8 causal prologue
# delay A/B, D = 256 backwardKeyValue late-DMA stamps.
set -o pipefail
OUT=gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py tests/test_plan_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "blockwise or kv8 or plan or golden or transposed" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/kv8_ab.py "C3 fp16,C3 bf16,D64 fp16,C2c fp16" --bw 64 > $OUT/ab_bw64.txt 2>&1 || exit $?
cat $OUT/ab_bw64.txt | sed 's/on-load plan.*//'
MFA_FWD_DELAY_SPLIT=8 timeout -k 10 200 python -u tools/ab_fwd.py MFA_FWD_DELAY=0,8 --cfg C2Q8 --rounds 12 > $OUT/ab_q8c_delay.json 2>&1 || exit $?
tail -1 $OUT/ab_q8c_delay.json
for v in bwd_stamps bwd_stamps_late bwd_stamps bwd_stamps_late; do
  timeout -k 10 120 tools/diag/$v 2 32 4096 256 > $OUT/$v.txt 2>&1 || exit $?
  echo "$v: $(grep bwd_kv $OUT/$v.txt)"
done
cat $OUT/bwd_stamps_late.txt
