#!/bin/bash
# GPU: batch-1 E5 encode latency + its kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e5b1; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/e5_b1_probe.py 2>&1 | tee gpurun_out/e5b1/probe.log | grep "E5 encode" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e5b1/trace -o t --output-format csv -- python3 -u tools/e5_b1_probe.py > gpurun_out/e5b1/tr.log 2>&1 || { tail -20 gpurun_out/e5b1/tr.log; exit 1; }
