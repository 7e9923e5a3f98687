#!/bin/bash
# K2a carried threshold (product) vs the per-list rule alone (variants/lib_nocarry.so): BM25 parity
# tests, per-kernel times (alternating), K2a PMC traffic, and the write split of the ablation build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/carry; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_filter.py tests/test_gpu_dropin.py tests/test_gpu_parallel.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -k "bm25 or hybrid or retrieve or filter" > gpurun_out/carry/tests.log 2>&1 || { tail -30 gpurun_out/carry/tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/carry/tests.log)"
for i in 1 2; do
  VARIANTS="variants/lib_orig.so variants/lib_carryonly.so variants/lib_blkonly.so" bash tools/k2_kprof.sh > gpurun_out/carry/kprof$i.txt 2>&1 || { tail -20 gpurun_out/carry/kprof$i.txt; exit 1; }
  cat gpurun_out/carry/kprof$i.txt
done
ONLY="bm25_B256" ROUND=carry bash tools/pmc_traffic.sh > gpurun_out/carry/pmc.txt 2>&1 || { tail -20 gpurun_out/carry/pmc.txt; exit 1; }
cat gpurun_out/pmc_traffic_carry.txt
DBG="${DBG:-0 1024 2048}" bash tools/k2a_wr.sh
