#!/bin/bash
# single-query retrieve() on the device chain: drop-in GPU tests, then the 10M e2e bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e2e4; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_engine.py tests/test_gpu_gemm.py -k "dropin or retrieve or e5 or attention or hybrid or graph or golden or expand or store" -x -q --timeout 300 --timeout-method thread > gpurun_out/e2e4/tests.log 2>&1 || { tail -30 gpurun_out/e2e4/tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/e2e4/tests.log)"
timeout -k 10 900 python -u bench.py --mode e2e --docs-per-gpu 10000000 --steps 10 --warmup 3 --out gpurun_out/e2e4/e2e.json > gpurun_out/e2e4/e2e.log 2>&1 || { tail -30 gpurun_out/e2e4/e2e.log; exit 1; }
grep -E "retrieve_batch calls" gpurun_out/e2e4/e2e.log | tail -2
