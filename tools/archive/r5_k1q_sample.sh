#!/bin/bash
# round 5: K1q (B = 256) seed-sample fraction in the headline step: 1/16 (product) vs 1/32 vs 1/8, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k1qs; export TMPDIR=/tmp
for r in 1 2; do
  for f in 16 32 8; do
    CM_K1Q_SAMPLE=$f timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/k1qs/bench_$f.log 2>&1 || { tail -20 gpurun_out/k1qs/bench_$f.log; exit 1; }
    grep "steps in" gpurun_out/k1qs/bench_$f.log | sed "s/^/frac=1\/$f /" | cut -c1-330
  done
done
