set -o pipefail
mkdir -p gpurun_out/p1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_forward_pipe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/p1/pytest.log 2>&1
rc=$?
tail -25 gpurun_out/p1/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_fwd.py MFA_FWD_PIPE=0,1 --cfg C3 --rounds 8 > gpurun_out/p1/ab_c3.txt 2>&1
rc=$?
tail -8 gpurun_out/p1/ab_c3.txt
exit $rc
