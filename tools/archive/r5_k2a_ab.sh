#!/bin/bash
# round 5: K2a pre-bound A/B (variants/lib_preb0.so = round-4 gather order, lib_preb1.so = pre-bound),
# standalone BM25 probe and headline-only bench, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k2a
for v in preb0 preb1; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 300 python -u tools/bm25_probe.py --paths 2 --reps 9 2>&1 | grep -E "docs=|workload" | sed "s/^/$v /"
done
for v in preb0 preb1 preb0 preb1; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 > gpurun_out/k2a/bench_$v.log 2>&1 || { tail -20 gpurun_out/k2a/bench_$v.log; exit 1; }
  grep "steps in" gpurun_out/k2a/bench_$v.log | sed "s/^/$v /" | cut -c1-420
done
