#!/bin/bash
# Round 6 closing check: the whole GPU suite, smoke(), the default bench (driver flags).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/final_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/final_pytest.log; exit 1; }
tail -2 gpurun_out/final_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/final_bench.json > gpurun_out/final_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/final_bench.log; exit 1; }
grep "\[bench\]" gpurun_out/final_bench.log | tail -12
