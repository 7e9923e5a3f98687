#!/bin/bash
# drop-in path after the host-glue change: drop-in GPU tests, then the 10M e2e bench with a host profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e2e2; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/e2e2/tests.log 2>&1 || { tail -30 gpurun_out/e2e2/tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/e2e2/tests.log)"
CM_E2E_PROFILE=1 timeout -k 10 900 python -u bench.py --mode e2e --docs-per-gpu 10000000 --steps 10 --warmup 3 --out gpurun_out/e2e2/e2e.json > gpurun_out/e2e2/e2e.log 2>&1 || { tail -30 gpurun_out/e2e2/e2e.log; exit 1; }
grep -E "retrieve_batch calls|q/s" gpurun_out/e2e2/e2e.log | tail -3
