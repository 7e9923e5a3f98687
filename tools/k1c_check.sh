#!/bin/bash
# GPU: dense parity tests, then K1c ablations at the bench shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/abl
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q -k "dense" --timeout 120 --timeout-method thread > gpurun_out/dense_tests.log 2>&1 || { tail -40 gpurun_out/dense_tests.log; exit 1; }
tail -2 gpurun_out/dense_tests.log
for d in ${DBG:-0 1 16 32}; do
  CM_DENSE_DEBUG=$d timeout -k 10 300 python tools/dense_probe.py --path 3 --reps 5 > gpurun_out/abl/c_$d.log 2>&1 || { tail -20 gpurun_out/abl/c_$d.log; exit 1; }
  echo "dbg=$d: $(tail -1 gpurun_out/abl/c_$d.log | cut -c1-150)"
done
