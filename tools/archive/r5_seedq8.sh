#!/bin/bash
# round 5: K1q seed pass in the gated step -- f16 K1c MINONLY over 1/16 (product: needs a whole CU, waits for
# K2a's blocks) vs the int8 K1q MINONLY in the shared 131 KiB footprint (beside K2a) over 1/8 and 1/16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/sq8; export TMPDIR=/tmp
for r in 1 2; do
  for v in f16 q8_8 q8_16; do
    env=""; [ $v = q8_8 ] && env="CM_K1Q_SEED=q8"; [ $v = q8_16 ] && env="CM_K1Q_SEED=q8 CM_K1Q_SAMPLE=16"
    env $env timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/sq8/bench_$v.log 2>&1 || { tail -20 gpurun_out/sq8/bench_$v.log; exit 1; }
    grep "steps in" gpurun_out/sq8/bench_$v.log | sed "s/^/$v /" | cut -c1-330
  done
done
