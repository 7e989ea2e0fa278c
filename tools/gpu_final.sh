#!/bin/bash
# Round-end evidence, part 1: the GPU parity suite (one process), the default bench line, smoke.
set -o pipefail
TAG=${1:-final}
bash tools/gpu_suite.sh $TAG || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -3 gpurun_out/$TAG/smoke.log
