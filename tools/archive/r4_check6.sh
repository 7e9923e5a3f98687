#!/bin/bash
# GPU: K1q band capacities (parity), drop-in e2e at 10M (retrieve_batch + single retrieve latency)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/c6; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_q8.py tests/test_gpu_dropin.py \
  "tests/test_gpu_scale.py::test_hybrid_10m_sample" > gpurun_out/c6/pytest.log 2>&1 || { tail -40 gpurun_out/c6/pytest.log; exit 1; }
tail -1 gpurun_out/c6/pytest.log
timeout -k 10 600 python -u bench.py --mode e2e --docs-per-gpu 10000000 --steps 5 --warmup 2 --e2e-latency-queries 32 \
  --out gpurun_out/c6/e2e_10m.json > gpurun_out/c6/e2e_10m.log 2>&1 || { tail -30 gpurun_out/c6/e2e_10m.log; exit 1; }
grep -E "steps in|retrieve\(\)|q/s" gpurun_out/c6/e2e_10m.log | cut -c1-250 | tail -8
