#!/bin/bash
# Round 6: masked key-phase prologue after moving the K/V loads behind the pre-pass: stamps,
# the sparse / backward parity tests, the block-sparse bench row.
set -o pipefail
OUT=gpurun_out/r06h
mkdir -p $OUT
timeout -k 10 120 tools/diag/bwd_stamps 1 16 4096 128 8 > $OUT/bwd_stamps_band8.txt 2>&1 || exit $?
cat $OUT/bwd_stamps_band8.txt
timeout -k 10 400 python -u -m pytest tests/test_sparse_gpu.py tests/test_backward_fast_gpu.py tests/test_backward_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 200 python -u tools/sparse_bwd_probe.py > $OUT/sparse_probe.txt 2>&1 || exit $?
cat $OUT/sparse_probe.txt
