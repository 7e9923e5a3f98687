#!/bin/bash
# K2a list heads in wave order (variants/lib_headsqg.so, -DCM_HEADS_QG=1) vs the product: BM25
# parity tests with the variant, per-kernel times (both, alternating), K2a PMC traffic (variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/heads; export TMPDIR=/tmp
CLASSMATE_HIP_LIB=$PWD/variants/lib_headsqg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread -k "bm25 or retrieve" > gpurun_out/heads/tests.log 2>&1 || { tail -30 gpurun_out/heads/tests.log; exit 1; }
echo "variant tests: $(tail -1 gpurun_out/heads/tests.log)"
VARIANTS="variants/lib_headsqg.so" bash tools/k2_kprof.sh > gpurun_out/heads/kprof.txt 2>&1 || { tail -20 gpurun_out/heads/kprof.txt; exit 1; }
cat gpurun_out/heads/kprof.txt
VARIANTS="variants/lib_headsqg.so" bash tools/k2_kprof.sh > gpurun_out/heads/kprof2.txt 2>&1 || { tail -20 gpurun_out/heads/kprof2.txt; exit 1; }
cat gpurun_out/heads/kprof2.txt
CLASSMATE_HIP_LIB=$PWD/variants/lib_headsqg.so ONLY="bm25_B256" ROUND=r03heads bash tools/pmc_traffic.sh > gpurun_out/heads/pmc.txt 2>&1 || { tail -20 gpurun_out/heads/pmc.txt; exit 1; }
cat gpurun_out/pmc_traffic_r03heads.txt
