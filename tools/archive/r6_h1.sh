#!/bin/bash
# Round 6 (late): K10_H1_6=2 (two row tiles before the mid-step barrier of the 96-row tiles) -- GEMM tests, step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
CLASSMATE_HIP_LIB=$PWD/variants/lib_h2.so timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/h2_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/h2_tests.log | tail -8
[ $rc -eq 0 ] || { tail -40 gpurun_out/h2_tests.log; exit 1; }
VARS="base h2 base h2 base h2" bash tools/r6_ab.sh
