#!/bin/bash
# Round 6 (late): fusion / select parity tests, then a same-box A/B of the headline step (variants/lib_*.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${T:-"tests/test_gpu_engine.py tests/test_gpu_q8.py tests/test_gpu_dropin.py"}
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread $T > gpurun_out/tail_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/tail_tests.log | tail -20
[ $rc -eq 0 ] || { tail -60 gpurun_out/tail_tests.log; exit 1; }
[ "${AB:-1}" = "1" ] && VARS=${VARS:-"base new base new"} bash tools/r6_ab.sh
