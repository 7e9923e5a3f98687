#!/bin/bash
# K10 tile A/B on the GPU box: accuracy tests and timings per forced tile (CM_K10_TILE), the product
# choice first.  GEMM shapes of the 256 x 24 query batch, then the whole fp32 E5 query encode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10t; export TMPDIR=/tmp
for t in ${TILES:-default 12x12 8x16}; do
  if [ "$t" = default ]; then unset CM_K10_TILE; else export CM_K10_TILE=$t; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread -k "linear or e5_query" > gpurun_out/k10t/test_$t.log 2>&1 || { echo "tile $t: tests FAILED"; tail -20 gpurun_out/k10t/test_$t.log; exit 1; }
  echo "tile $t: $(tail -1 gpurun_out/k10t/test_$t.log)"
  K10_E5=1 timeout -k 10 300 python -u tools/k10_probe.py > gpurun_out/k10t/probe_$t.log 2>&1 || { tail -20 gpurun_out/k10t/probe_$t.log; exit 1; }
  grep -E "K10|E5 query encode B=256 S=24 fp32 K10" gpurun_out/k10t/probe_$t.log | sed "s/^/  [$t] /"
done
