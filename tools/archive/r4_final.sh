#!/bin/bash
# GPU: round-4 final check on the current tree: GPU suite + smoke, default bench, headline-only kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/fin; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/fin/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/fin/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || { tail -20 gpurun_out/fin/smoke.log; exit 1; }
tail -1 gpurun_out/fin/smoke.log
timeout -k 10 600 python -u bench.py --out gpurun_out/fin/bench_default.json > gpurun_out/fin/bench_default.log 2>&1 || { tail -30 gpurun_out/fin/bench_default.log; exit 1; }
tail -1 gpurun_out/fin/bench_default.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/fin/trace -o hl --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/fin/bench_hl.json > gpurun_out/fin/bench_hl.log 2>&1 || { tail -30 gpurun_out/fin/bench_hl.log; exit 1; }
grep "steps in" gpurun_out/fin/bench_hl.log | cut -c1-300
