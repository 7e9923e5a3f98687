#!/bin/bash
# round 5: headline kernel trace of the current tree -> gpurun_out/trace/hl (step timeline via tools/trace_step.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/trace; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace/hl -o hl --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/trace/bench.log 2>&1 || { tail -30 gpurun_out/trace/bench.log; exit 1; }
grep "steps in" gpurun_out/trace/bench.log | cut -c1-200
python3 tools/trace_step.py gpurun_out/trace/hl/hl_kernel_trace.csv dense_q8_scan_kernel 15 | grep -v "linear_f16x3\|short_att\|add_layernorm" | tail -22
