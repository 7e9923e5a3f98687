#!/bin/bash
# GPU: ablations + PMC passes for the two dominant kernels (K1b dense, K2 BM25) at the bench shape.
#   tools/perf_probe.sh            -> gpurun_out/perf/*.log, gpurun_out/pmc_{dense,bm25}.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/perf; export TMPDIR=/tmp
for d in ${K2_DBG:-0 1 2 3}; do
  CM_BM25_DEBUG=$d timeout -k 10 300 python tools/bm25_probe.py > gpurun_out/perf/bm25_$d.log 2>&1 || { tail -20 gpurun_out/perf/bm25_$d.log; exit 1; }
  echo "bm25 dbg=$d: $(tail -1 gpurun_out/perf/bm25_$d.log)"
done
head -1 gpurun_out/perf/bm25_0.log
for d in ${K1_DBG:-0 1}; do
  CM_DENSE_DEBUG=$d timeout -k 10 300 python tools/dense_probe.py > gpurun_out/perf/dense_$d.log 2>&1 || { tail -20 gpurun_out/perf/dense_$d.log; exit 1; }
  echo "dense dbg=$d: $(tail -1 gpurun_out/perf/dense_$d.log)"
done
if [ "${PMC:-1}" = "1" ]; then
  bash tools/pmc.sh bm25 bm25_range_kernel -- python3 tools/bm25_probe.py --reps 2 || exit 1
  bash tools/pmc.sh dense dense_f16x3_kernel -- python3 tools/dense_probe.py --reps 2 || exit 1
fi
