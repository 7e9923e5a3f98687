#!/bin/bash
# round 5: wide re-rank with overflowed-group re-scan -- q8 + certificate tests, then the duplicate-cluster leg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/wide2; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_q8.py tests/test_gpu_engine.py -k "q8 or certificate or Q8" > gpurun_out/wide2/pytest.log 2>&1 || { tail -40 gpurun_out/wide2/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/wide2/pytest.log | tail -2
timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 --e5-other-leg 0 --ingest-leg 0 --cpu-baseline 0 --out gpurun_out/wide2/bench.json > gpurun_out/wide2/bench.log 2>&1 || { tail -20 gpurun_out/wide2/bench.log; exit 1; }
grep -E "steps in|c4_dense|c2p|c4_dup" gpurun_out/wide2/bench.log | cut -c1-250
