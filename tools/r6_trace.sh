#!/bin/bash
# Round 6: headline-step kernel trace (no side legs) -> one step's timeline (tools/trace_step.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/trace6; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace6/hl -o hl --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/trace6/bench.log 2>&1 || { tail -30 gpurun_out/trace6/bench.log; exit 1; }
grep "steps in" gpurun_out/trace6/bench.log | cut -c1-200
f=$(find gpurun_out/trace6/hl -name '*kernel_trace.csv' | head -1); cp "$f" gpurun_out/trace6/kernel_trace.csv
