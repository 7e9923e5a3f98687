#!/bin/bash
# round-3 perf survey on the GPU box: K10 GEMMs (kernel trace), the fp32 E5 encode per kernel, the
# BM25 pruned search per kernel (product library) and K2a/K2b PMC traffic.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/k10_prof.sh > gpurun_out/r3s_k10.txt 2>&1 || { tail -20 gpurun_out/r3s_k10.txt; exit 1; }
tail -16 gpurun_out/r3s_k10.txt
bash tools/e5_kprof.sh > gpurun_out/r3s_e5.txt 2>&1 || { tail -20 gpurun_out/r3s_e5.txt; exit 1; }
head -30 gpurun_out/r3s_e5.txt
VARIANTS=" " bash tools/k2_kprof.sh > gpurun_out/r3s_bm25.txt 2>&1 || { tail -20 gpurun_out/r3s_bm25.txt; exit 1; }
cat gpurun_out/r3s_bm25.txt
ONLY="bm25_B256 bm25b_B256" ROUND=r03 bash tools/pmc_traffic.sh > gpurun_out/r3s_pmc.txt 2>&1 || { tail -20 gpurun_out/r3s_pmc.txt; exit 1; }
cat gpurun_out/pmc_traffic_r03.txt
DOCS=1000000 bash tools/mgpu_rehearsal.sh > gpurun_out/r3s_mgpu.txt 2>&1 || { tail -20 gpurun_out/r3s_mgpu.txt; exit 1; }
cat gpurun_out/r3s_mgpu.txt
