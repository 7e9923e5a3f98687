#!/bin/bash
# drop-in path after the host changes + masked split attention: attention / E5 / drop-in GPU tests,
# then the 10M e2e bench (no profiler in the timed loop)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e2e3; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_dropin.py tests/test_gpu_engine.py -k "attention or e5 or linear or plane or retrieve or dropin or hybrid or graph" -x -q --timeout 300 --timeout-method thread > gpurun_out/e2e3/tests.log 2>&1 || { tail -30 gpurun_out/e2e3/tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/e2e3/tests.log)"
grep -E "masked attention|attention S=" gpurun_out/e2e3/tests.log | head -12
timeout -k 10 900 python -u bench.py --mode e2e --docs-per-gpu 10000000 --steps 10 --warmup 3 --out gpurun_out/e2e3/e2e.json > gpurun_out/e2e3/e2e.log 2>&1 || { tail -30 gpurun_out/e2e3/e2e.log; exit 1; }
grep -E "retrieve_batch calls" gpurun_out/e2e3/e2e.log | tail -2
