#!/bin/bash
# CPU sanitizer run: the oracle and the library's host code (the
# C-ABI layer and the plan path, which run without a GPU) under AddressSanitizer and
# UndefinedBehavior checks (trap mode), driven by the CPU tests that exercise them.
#   make -C oracle asan && make -C metal-flash-attention-plus_amd asan   (once)
#   bash tools/asan_check.sh [pytest args...]
set -o pipefail
cd "$(dirname "$0")/.."
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
make -s -C oracle asan || exit 1
[ -f metal-flash-attention-plus_amd/build_asan/libmfa_amd_asan.so ] || make -s -j8 -C metal-flash-attention-plus_amd asan || exit 1
SEL=${@:-tests/test_oracle.py tests/test_plan.py tests/test_golden.py tests/test_abi.py tests/test_manifest.py}
# detect_leaks=0: CPython and torch keep their allocations to exit.  The Python interpreter and
# torch are not instrumented; only the preloaded runtime's interceptors see their calls.
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
MFA_LIB=$PWD/metal-flash-attention-plus_amd/build_asan/libmfa_amd_asan.so \
MFA_ORACLE_LIB=$PWD/oracle/_asan/libmfa_oracle.so \
  python -m pytest $SEL -q -m "not gpu" -p no:cacheprovider
