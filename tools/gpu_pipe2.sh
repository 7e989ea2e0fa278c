set -o pipefail
mkdir -p gpurun_out/p2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_forward_pipe_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p2/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/p2/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/diag/pipe_abl 16 8192 s,0,s,0 > gpurun_out/p2/abl.txt 2>&1
rc=$?
cat gpurun_out/p2/abl.txt
exit $rc
