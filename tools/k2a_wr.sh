#!/bin/bash
# K2a write-traffic split (ablation build variants/lib_abl.so; results NOT valid): PMC WRITE_SIZE
# with the list sentinels (1024), list entries (2048), need bytes (4096) switched off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in ${DBG:-0 1024 2048 4096 7168}; do
  CLASSMATE_HIP_LIB=$PWD/variants/lib_abl.so CM_BM25_DEBUG=$d ONLY="bm25_B256" ROUND=wr$d bash tools/pmc_traffic.sh > gpurun_out/wr_$d.log 2>&1 || { tail -20 gpurun_out/wr_$d.log; exit 1; }
  echo "dbg=$d $(cat gpurun_out/pmc_traffic_wr$d.txt)"
done
