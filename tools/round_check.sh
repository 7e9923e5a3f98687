#!/bin/bash
# GPU: what the driver runs at round end (pytest -m gpu, smoke, bench) + a rocprofv3 summary of the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep "\[bench\] 10" gpurun_out/bench.log; tail -1 gpurun_out/bench.log > gpurun_out/bench.json
bash tools/bench_prof.sh > gpurun_out/bench_prof_summary.txt 2>&1 || { tail -5 gpurun_out/bench_prof_summary.txt; exit 1; }
head -3 gpurun_out/bench_prof_summary.txt
