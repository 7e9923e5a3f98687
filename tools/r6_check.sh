#!/bin/bash
# Round 6: the new tests first (verbose), then the whole GPU suite, then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
NEW=${NEW:-"tests/test_gpu_multidev.py tests/test_gpu_threads.py tests/test_gpu_dropin.py::test_vector_store_cold_open_replaces_old_metadata"}
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread $NEW > gpurun_out/new.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/new.log | tail -40
[ $rc -eq 0 ] || { tail -60 gpurun_out/new.log; exit 1; }
if [ "${FULL:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
  grep "\[bench\]" gpurun_out/bench.log | tail -20
fi
