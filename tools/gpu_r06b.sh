#!/bin/bash
# Round 6: re-check the new quantised-backward / graph tests and the INT8 tests, C2 stamps of the
# mirrored and stream kernels, INT8 bias-tile A/B at C3.
set -o pipefail
OUT=gpurun_out/r06b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py tests/test_forward_stream_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 tools/diag/fwd_stamps 16 4096 1 p 400 > $OUT/fwd_stamps_c2.txt 2>&1 || exit $?
cat $OUT/fwd_stamps_c2.txt
timeout -k 10 120 tools/diag/stream_stamps 16 4096 128 > $OUT/stream_stamps_c2.txt 2>&1 || exit $?
cat $OUT/stream_stamps_c2.txt
timeout -k 10 200 python -u tools/ab_fwd.py MFA_I8_BIAS=0,1 --cfg C3I8 --rounds 10 > $OUT/ab_i8_bias.json 2>&1 || exit $?
cat $OUT/ab_i8_bias.json
exit $rc
