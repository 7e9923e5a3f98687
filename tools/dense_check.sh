#!/bin/bash
# GPU: dense parity tests, then every scan path at the bench shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q -k "dense" --timeout 120 --timeout-method thread > gpurun_out/dense_tests.log 2>&1 || { tail -40 gpurun_out/dense_tests.log; exit 1; }
tail -2 gpurun_out/dense_tests.log
for p in ${PATHS:-3 2}; do
  timeout -k 10 300 python tools/dense_probe.py --path $p > gpurun_out/dprobe_$p.log 2>&1 || { tail -20 gpurun_out/dprobe_$p.log; exit 1; }
  echo "path $p: $(tail -1 gpurun_out/dprobe_$p.log)"
done
