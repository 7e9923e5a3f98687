#!/bin/bash
# round 5 GPU check: full GPU suite + smoke + default bench (driver-equivalent line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/chk; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/chk/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/chk/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk/smoke.log 2>&1 || { tail -20 gpurun_out/chk/smoke.log; exit 1; }
tail -1 gpurun_out/chk/smoke.log
timeout -k 10 600 python -u bench.py --out gpurun_out/chk/bench_default.json > gpurun_out/chk/bench_default.log 2>&1 || { tail -30 gpurun_out/chk/bench_default.log; exit 1; }
grep -E "steps in|c2p|c4_dense|c2_dense|ingest|E5 leg" gpurun_out/chk/bench_default.log | cut -c1-400
