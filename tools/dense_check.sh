#!/bin/bash
# GPU: dense parity tests, then both K1 paths at the bench shape.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py -x -q -k "dense" > gpurun_out/dense_tests.log 2>&1 || { tail -40 gpurun_out/dense_tests.log; exit 1; }
tail -2 gpurun_out/dense_tests.log
for p in f16x3 f32; do
  CM_DENSE_PATH=$p timeout -k 10 300 python tools/dense_probe.py > gpurun_out/dprobe_$p.log 2>&1 || { tail -20 gpurun_out/dprobe_$p.log; exit 1; }
  echo "$p $(tail -1 gpurun_out/dprobe_$p.log)"
done
