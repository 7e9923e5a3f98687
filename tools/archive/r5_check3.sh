#!/bin/bash
# round 5: the large-batch geometry test + the dense q8/scale suites on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/c3; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_q8.py > gpurun_out/c3/pytest_q8.log 2>&1 || { tail -40 gpurun_out/c3/pytest_q8.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/c3/pytest_q8.log | tail -20
