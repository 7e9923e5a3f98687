#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for d in 0 1; do
  CM_DENSE_DEBUG=$d timeout -k 10 300 python tools/dense_probe.py > gpurun_out/dab_$d.log 2>&1 || { tail -20 gpurun_out/dab_$d.log; exit 1; }
  echo "dbg=$d $(tail -1 gpurun_out/dab_$d.log)"
done
