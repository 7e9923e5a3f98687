#!/bin/bash
# Round 6 (late): K10 96 x 288 QKV tile -- GEMM / E5 parity tests, then the step A/B against the 96 x 192 tile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/t288_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/t288_tests.log | tail -8
[ $rc -eq 0 ] || { tail -40 gpurun_out/t288_tests.log; exit 1; }
ENVS="t288 t192=CM_K10_T288=0" REPS=3 bash tools/r6_env_ab.sh
