#!/bin/bash
# GPU: small batches on K1q (forced, --path 5) vs the automatic K1s stream scan, 10M x 768, k = 24 and 10
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/sq8
for rep in 1 2; do for b in 1 16 64; do for p in 0 5; do
  timeout -k 10 300 python tools/dense_probe.py --batch $b --k 24 --path $p --reps 9 > gpurun_out/sq8/p.log 2>&1 || { tail -20 gpurun_out/sq8/p.log; exit 1; }
  grep docs= gpurun_out/sq8/p.log | sed "s/^/path=$p /" | cut -c1-150 | tee -a gpurun_out/sq8/ab.txt
done; done; done
